"""The camera trunk's M = 128 token GEMMs (forward, dX, dW shapes): split-K over few tiles vs the
unsplit plans (COMET_GEMM_NO_SMALLSPLIT=1).

    python tools/small_gemm_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from comet_amd import ops  # noqa: E402
from tile_bench import timed  # noqa: E402

SHAPES = [  # (M, N, K, layout_a, layout_b, out dtype)
    (128, 768, 768, 0, 0, torch.bfloat16), (128, 3072, 768, 0, 0, torch.bfloat16), (128, 768, 3072, 0, 0, torch.float32),
    (128, 768, 768, 0, 1, torch.bfloat16), (128, 768, 3072, 0, 1, torch.bfloat16),
    (768, 768, 128, 1, 1, torch.float32), (768, 3072, 128, 1, 1, torch.float32), (3072, 768, 128, 1, 1, torch.float32),
]


def main():
    torch.manual_seed(0)
    for M, N, K, la, lb, odt in SHAPES:
        A = torch.randn(*((M, K) if la == 0 else (K, M)), device="cuda").to(torch.bfloat16)
        B = torch.randn(*((N, K) if lb == 0 else (K, N)), device="cuda").to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=odt)
        fn = lambda: ops.gemm_raw(A, B, C, m=M, n=N, k=K, layout_a=la, lda=A.stride(0), layout_b=lb, ldb=B.stride(0), ldc=N)
        t_new = timed(fn)
        fn()
        ref = C.float().clone()
        os.environ["COMET_GEMM_NO_SMALLSPLIT"] = "1"
        t_old = timed(fn)
        fn()
        os.environ.pop("COMET_GEMM_NO_SMALLSPLIT")
        err = ((C.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"M{M} N{N} K{K} L{la}{lb} {str(odt)[6:]}: new {t_new:6.1f} us  old {t_old:6.1f} us  rel diff {err:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
