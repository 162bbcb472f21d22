"""Row-LN GEMM (comet_gemm_rowln) vs the residual GEMM + LayerNorm kernels it replaces, on the
tracker's update-former shapes (out_proj K = 384 -> norm2; fc2 K = 1536 -> next norm1 dual (+ ctx)).

    python tools/rowln_bench.py            (set COMET_ROWLN_HALF=1 for the half-height tiles)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

SHAPES = [  # (M, N, K, mode)
    (65536, 384, 384, "norm2"), (65536, 384, 1536, "dual"), (65536, 384, 1536, "dual_ctx"),
    (8192, 384, 384, "norm2"), (8192, 384, 1536, "dual_ctx"), (65536, 256, 256, "norm2"), (65536, 256, 1024, "dual"),
]


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
    for M, N, K, mode in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        b = torch.rand(N, device="cuda")
        r = torch.rand(M, N, device="cuda")
        zw, zb = torch.rand(N, device="cuda"), torch.rand(N, device="cuda")
        raw = mode == "norm2"
        z = (zw, zb, 1e-5) if mode == "dual_ctx" else None

        def fused():
            ops.linear_rowln(x, w, b, r, raw=raw, y16_eps=1e-6, z=z)

        def separate():
            c = ops.linear(x, w, bias=b, resid=r, out_dtype=torch.float32)
            if z is not None:
                ops.layernorm(c, zw, zb, eps=1e-5, out_dtype=torch.bfloat16)
            if raw:
                ops.layernorm(c, eps=1e-6, out_dtype=torch.bfloat16)
            else:
                ops.layernorm(c, eps=1e-6, out_dtype=torch.float32, dual=True)

        tf, ts = timed(fused), timed(separate)
        nbytes = 2 * M * K + 2 * N * K + 4 * M * N * 2 + 2 * M * N * (1 + (z is not None))
        extra = ""
        if os.environ.get("COMET_ROWLN_AB"):  # B arm: the env var COMET_ROWLN_AB names, set to 1
            os.environ[os.environ["COMET_ROWLN_AB"]] = "1"
            tb = timed(fused)
            del os.environ[os.environ["COMET_ROWLN_AB"]]
            extra = f"   {os.environ['COMET_ROWLN_AB']}: {tb:7.1f} us ({nbytes / tb / 1e6:.2f} TB/s)"
        print(f"M{M} N{N} K{K} {mode:9s} fused {tf:7.1f} us ({nbytes / tf / 1e6:.2f} TB/s, "
              f"{2 * M * N * K / tf / 1e6:.0f} TF/s)   gemm+LN {ts:7.1f} us{extra}", flush=True)


if __name__ == "__main__":
    main()
