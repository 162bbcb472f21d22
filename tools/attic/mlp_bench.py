"""Fused update-former MLP (comet_mlp_rowln) vs the unfused pair it replaces (fc1 GELU GEMM +
fc2 row-LN GEMM), on the tracker's shapes.   python tools/mlp_bench.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

SHAPES = [(65536, 384, 1536, "dual_ctx"), (65536, 384, 1536, "dual"), (65536, 256, 1024, "dual"),
          (16384, 384, 1536, "dual"), (8192, 384, 1536, "dual")]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    for M, C, Hd, mode in SHAPES:
        x = ((torch.rand(M, C, device="cuda") * 2 - 1)).to(torch.bfloat16)
        w1 = ((torch.rand(Hd, C, device="cuda") * 2 - 1) * C ** -0.5).to(torch.bfloat16)
        w2 = ((torch.rand(C, Hd, device="cuda") * 2 - 1) * Hd ** -0.5).to(torch.bfloat16)
        b1, b2 = torch.rand(Hd, device="cuda"), torch.rand(C, device="cuda")
        r = torch.rand(M, C, device="cuda")
        z = (torch.rand(C, device="cuda"), torch.rand(C, device="cuda"), 1e-5) if mode == "dual_ctx" else None

        def fused():
            ops.mlp_rowln(x, w1, b1, w2, b2, r, raw=False, y16_eps=1e-6, z=z)

        def unfused():
            h = ops.linear(x, w1, bias=b1, act=1, out_dtype=torch.bfloat16)
            ops.linear_rowln(h, w2, b2, r, raw=False, y16_eps=1e-6, z=z)

        tf, tu = timed(fused), timed(unfused)
        fl = 4.0 * M * C * Hd
        print(f"M{M} C{C} H{Hd} {mode:8s} fused {tf:7.1f} us ({fl / tf / 1e6:5.0f} TF/s)  unfused {tu:7.1f} us "
              f"({fl / tu / 1e6:5.0f} TF/s)  saved {tu - tf:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
