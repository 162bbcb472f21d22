"""ORACLE / TEST INFRASTRUCTURE ONLY — counter-based PRNG for parameters and inputs.

Only tests/, tools/gen_golden.py, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package. The same generator builds the weights on the generator side (reference
model, this container) and on the checker side (oracle + HIP path), so golden fixtures only
have to store seeds and outputs, never the 1 GB of weights.

value(seed, name, i) = 2 * (splitmix64(fnv1a64(name) ^ seed*GOLDEN + i) >> 40) / 2^24 - 1
"""
import numpy as np
import torch

_M64 = (1 << 64) - 1


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & _M64
    return h


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed: int, name: str, shape) -> np.ndarray:
    """float32 array in [-1, 1) with 24-bit resolution."""
    n = int(np.prod(shape)) if len(shape) else 1
    base = (fnv1a64(name) ^ ((seed * 0x9E3779B97F4A7C15) & _M64)) & _M64
    with np.errstate(over="ignore"):
        z = _splitmix64(np.arange(n, dtype=np.uint64) + np.uint64(base))
    u = (z >> np.uint64(40)).astype(np.float64) * (2.0 / (1 << 24)) - 1.0
    return u.astype(np.float32).reshape(shape)


def normal_like(seed: int, name: str, shape) -> np.ndarray:
    """Approximately N(0,1): sum of 4 uniforms, variance matched (deterministic, cheap)."""
    acc = np.zeros(shape, dtype=np.float64)
    for j in range(4):
        acc += uniform(seed, f"{name}#{j}", shape)
    return (acc * np.sqrt(3.0 / 4.0)).astype(np.float32)


_TOKEN_SCALE = {
    "cls_token": 0.1, "register_tokens": 0.1, "mask_token": 0.1, "pos_embed": 0.1,
    "pose_token": 0.1, "virual_tracks": 1.0,
}


def param_value(seed: int, name: str, shape) -> torch.Tensor:
    """Deterministic initial value of parameter `name` (state_dict key) of a given shape.

    rules: >=2-D weights U(-1,1)/sqrt(fan_in); 1-D `*.weight` (norm affine) 1 + 0.1U;
    1-D biases 0.05U; LayerScale gammas 0.1 + 0.05U; token/embedding tables by _TOKEN_SCALE;
    0-D / 1-element scalars 0.5 + 0.1U.
    """
    shape = tuple(shape)
    u = uniform(seed, name, shape)
    leaf = name.split(".")[-1]
    if leaf in _TOKEN_SCALE:
        v = u * _TOKEN_SCALE[leaf]
    elif leaf == "gamma":
        v = 0.1 + 0.05 * u
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = u / np.sqrt(fan_in)
    elif len(shape) == 0 or (len(shape) == 1 and shape[0] == 1 and "bias" not in leaf):
        v = 0.5 + 0.1 * u
    elif leaf.endswith("weight"):
        v = 1.0 + 0.1 * u
    else:
        v = 0.05 * u
    return torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))


def make_state_dict(seed: int, shapes: dict) -> dict:
    """shapes: name -> shape (e.g. {k: v.shape for k, v in model.state_dict().items()})."""
    return {k: param_value(seed, k, s) for k, s in shapes.items()}
