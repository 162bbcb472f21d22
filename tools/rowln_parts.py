"""Where a row-LN GEMM's time goes: the fused kernel against the same GEMM without the LN epilogue
(f32 + residual, and plain bf16 output) on the tracker's fc2 / out_proj shapes.

    python tools/rowln_parts.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402


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
    for M, N, K in [(65536, 384, 1536), (65536, 384, 384), (65536, 256, 1024)]:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        b = torch.rand(N, device="cuda")
        r = torch.rand(M, N, device="cuda")
        zw, zb = torch.rand(N, device="cuda"), torch.rand(N, device="cuda")
        fl = 2.0 * M * N * K
        arms = {
            "rowln dual+ctx": lambda: ops.linear_rowln(x, w, b, r, raw=False, y16_eps=1e-6, z=(zw, zb, 1e-5)),
            "rowln raw+y16": lambda: ops.linear_rowln(x, w, b, r, raw=True, y16_eps=1e-6),
            "gemm f32+res": lambda: ops.linear(x, w, bias=b, resid=r, out_dtype=torch.float32),
            "gemm bf16": lambda: ops.linear(x, w, bias=b, out_dtype=torch.bfloat16),
        }
        for name, fn in arms.items():
            us = timed(fn)
            plan = tuple(ops._PLAN) if name.startswith("gemm") else ""
            print(f"M {M} N {N} K {K} {name:16s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s {plan}", flush=True)


if __name__ == "__main__":
    main()
