"""Per-tile fixed cost vs per-k-tile cost of the forward GEMM kernels: time M x N x K for a K sweep."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402


def bench(fn, iters=10):
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


M, N = 74368, 3072
for odt in (torch.bfloat16, torch.float32):
    for K in (64, 128, 256, 512, 768, 1536, 3072):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=odt)
        row = []
        for env in (None, "COMET_GEMM_NO_PP"):
            if env:
                os.environ[env] = "1"
            row.append(bench(lambda: ops.linear(x, w, out=out, out_dtype=odt)))
            if env:
                del os.environ[env]
        row.append(bench(lambda: torch.matmul(x, w.t())))
        print(f"{str(odt)[6:]:>8} K {K:5d}: w4 {row[0]:8.1f} us  big {row[1]:8.1f} us  torch {row[2]:8.1f} us", flush=True)
