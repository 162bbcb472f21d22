"""Persistent GEMM tile choice on the step's plain-GEMM shapes: each tile instance of the w4 kernel
(COMET_PP_TILE override) timed with HIP events, plus a check that every tile gives the same result.

    python tools/tile_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import _lib as L  # noqa: E402
from comet_amd import ops  # noqa: E402

SHAPES = [  # (M, N, K, act, out dtype, residual)  -- profiles/r02_v3/gemm_shapes.txt
    (8192, 1536, 384, L.ACT_GELU, torch.bfloat16, False),
    (8192, 1152, 384, L.ACT_NONE, torch.bfloat16, False),
    (8192, 768, 384, L.ACT_NONE, torch.bfloat16, False),
    (8192, 384, 384, L.ACT_NONE, torch.bfloat16, False),
    (65536, 1152, 384, L.ACT_NONE, torch.bfloat16, False),
    (65536, 1536, 384, L.ACT_GELU, torch.bfloat16, False),
    (65536, 768, 384, L.ACT_NONE, torch.bfloat16, False),
    (65536, 1024, 256, L.ACT_GELU, torch.bfloat16, False),
    (65536, 768, 256, L.ACT_NONE, torch.bfloat16, False),
    (74368, 3072, 768, L.ACT_GELU, torch.bfloat16, False),
    (65536, 1536, 384, L.ACT_NONE, torch.bfloat16, False),  # the GELU shapes without the activation:
    (74368, 3072, 768, L.ACT_NONE, torch.bfloat16, False),  # the epilogue's share
    (74368, 2304, 768, L.ACT_NONE, torch.bfloat16, False),
    (74368, 768, 3072, L.ACT_NONE, torch.float32, True),
    (74368, 768, 768, L.ACT_NONE, torch.float32, True),
]
TILES = ["256x256", "128x256", "128x384", "64x384"]


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
    torch.manual_seed(0)
    for M, N, K, act, odt, res in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        b = torch.rand(N, device="cuda")
        r = torch.rand(M, N, device="cuda") if res else None
        out = torch.empty(M, N, device="cuda", dtype=odt)
        fn = lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out)
        line, ref = [], None
        for t in TILES:
            os.environ["COMET_PP_TILE"] = t
            us = timed(fn)
            fn()
            torch.cuda.synchronize()
            same = "" if ref is None else ("=" if torch.equal(out, ref) else "DIFF")
            if ref is None:
                ref = out.clone()
            line.append(f"{t} {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.1f} TF/s {same}")
        os.environ.pop("COMET_PP_TILE")
        base = timed(fn)
        print(f"M{M} N{N} K{K} act{act} {str(odt)[6:]}{' res' if res else ''}: default {base:7.1f} us | " + " | ".join(line),
              flush=True)


if __name__ == "__main__":
    main()
