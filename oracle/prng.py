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
    if ".updateformer.flow_head." in name:
        # parity-friendly damping: random-weight tracker iterations are chaotic (an fp32 ulp at
        # iteration 0 grows ~100x per iteration); small coordinate/feature updates keep the
        # reference, the oracle and the HIP path comparable after 4-6 iterations.
        v = v * FLOW_HEAD_DAMP
    return torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))


FLOW_HEAD_DAMP = 0.01


def make_state_dict(seed: int, shapes: dict) -> dict:
    """shapes: name -> shape (e.g. {k: v.shape for k, v in model.state_dict().items()})."""
    return {k: param_value(seed, k, s) for k, s in shapes.items()}


def synthetic_batch(seed: int, B: int, T: int, H: int, W: int, N: int):
    """Synthetic inputs of SURVEY.md §8(d): images ~N(0,1) (post-normalisation distribution),
    kp0 ~ U[0, W-1]^2 broadcast over T, unit quaternions (w >= 0), T_uvz = (U[270,370],
    U[190,290], U[5,15]), T_xyz ~ N(0,1), focal 268.44, ratio 0.5 (float64, as collated)."""
    img = torch.from_numpy(normal_like(seed, "images", (B, T, 3, H, W)))
    kp = (uniform(seed, "kp0", (B, N, 2)) + 1.0) * 0.5 * np.float32(W - 1)
    tracks = torch.from_numpy(kp).unsqueeze(1).expand(B, T, N, 2).contiguous()
    q = normal_like(seed, "quat", (B * T, 4)).astype(np.float64)
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    q[q[:, 0] < 0] *= -1
    u = uniform(seed, "uvz", (B * T, 3))
    uvz = np.stack([320 + 50 * u[:, 0], 240 + 50 * u[:, 1], 10 + 5 * u[:, 2]], -1).astype(np.float32)
    gt = {
        "R": torch.from_numpy(q.astype(np.float32)),
        "T_uvz": torch.from_numpy(uvz),
        "T": torch.from_numpy(normal_like(seed, "txyz", (B * T, 3))),
        "focal_length": torch.full((B * T, 2), 268.44),
        "principal_point": torch.zeros(B * T, 2),
        "ratio": torch.tensor([0.5], dtype=torch.float64),
    }
    return img, tracks, gt


def loop_batches(seed, B=1, T=4, H=128, W=128, N=256, steps=2):
    """Inputs of the loop golden (tools/gen_golden.py --loop, tests/test_loop_gpu.py): `steps`
    batches in process_spark_data2's dict layout (train_util.py:637-667; frames and GT from
    synthetic_batch), an all-true first-frame mask, and the N fixed frame-0 keypoints a SuperPoint
    stub returns ("kp0"; all inside the mask, so filter_and_pad takes its RNG-free branch when
    N = min_required = track_num = 256)."""
    out = []
    for st in range(steps):
        img, _, gt = synthetic_batch(seed + 100 * st, B, T, H, W, 16)
        g = torch.Generator().manual_seed(seed + 100 * st + 7)
        kp = torch.rand(N, 2, generator=g) * (W - 1)
        out.append({"images": img, "T": gt["T"].reshape(B, T, 3), "T_uvz": gt["T_uvz"].reshape(B, T, 3),
                    "R": gt["R"].reshape(B, T, 4), "ratio": gt["ratio"], "fl": gt["focal_length"].reshape(B, T, 2),
                    "pp": gt["principal_point"].reshape(B, T, 2), "seq_name": [f"seq{st}"],
                    "first_mask": torch.ones(B, H, W, dtype=torch.bool), "kp0": kp})
    return out
