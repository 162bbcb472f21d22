"""Microbenchmark of comet_attention_fwd / _bwd on the COMET step's attention shapes.

    python tools/attn_bench.py > gpurun_out/attn_bench.txt

TFLOP/s counts 4*B*H*Lq*Lk*D (forward) and 10*B*H*Lq*Lk*D (backward) at the true head_dim.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

# (name, B, H, Lq, Lk, D, backward?)
SHAPES = [
    ("dino self", 128, 12, 581, 581, 64, False),
    ("head self", 128, 8, 577, 577, 96, True),
    ("head cross", 8, 8, 8655, 577, 96, True),
    ("tracker p2v", 128, 8, 512, 64, 48, False),
    ("tracker v2p", 128, 8, 64, 512, 48, False),
    ("tracker virt", 128, 8, 64, 64, 48, False),
    ("trunk", 8, 8, 16, 16, 96, True),
    ("T_P cross", 128, 8, 1, 512, 96, True),
    ("long T64 768", 4, 12, 64 * 37 * 37 // 64 + 1, 64 * 37 * 37 // 64 + 1, 64, False),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for name, B, H, Lq, Lk, D, bwd in SHAPES:
        C = H * D
        q = torch.randn(B, Lq, C, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, Lk, C, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, Lk, C, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: ops.attention(q, k, v, H, D ** -0.5, lse=True))
        fl = 4.0 * B * H * Lq * Lk * D
        line = f"{name:14s} B{B:4d} H{H:3d} Lq{Lq:5d} Lk{Lk:5d} D{D:3d}  fwd {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s"
        if os.environ.get("COMET_ATTN_AB"):  # both forward kernels forced on the same shape
            for var, tag in (("COMET_ATTN_FWD16", "16x16"), ("COMET_ATTN_FWD32", "32x32")):
                os.environ[var] = "1"
                msx = timeit(lambda: ops.attention(q, k, v, H, D ** -0.5, lse=True))
                del os.environ[var]
                line += f" ({tag}: {msx * 1e3:7.1f} us {fl / msx / 1e9:6.1f})"
        if bwd:
            o, lse = ops.attention(q, k, v, H, D ** -0.5, lse=True)
            do = torch.randn_like(o)
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            msb = timeit(lambda: ops.attention_bwd(q, k, v, o, lse, do, H, D ** -0.5, dq, dk, dv))
            line += f"  bwd {msb * 1e3:8.1f} us {2.5 * fl / msb / 1e9:7.1f} TF/s"
            if os.environ.get("COMET_ATTN_AB"):  # the 16x16x32 backward kernels
                os.environ["COMET_ATTN_BWD16"] = "1"
                msb16 = timeit(lambda: ops.attention_bwd(q, k, v, o, lse, do, H, D ** -0.5, dq, dk, dv))
                del os.environ["COMET_ATTN_BWD16"]
                line += f" (16x16: {msb16 * 1e3:8.1f} us {2.5 * fl / msb16 / 1e9:7.1f})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
