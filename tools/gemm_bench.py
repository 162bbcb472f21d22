"""Microbenchmark of comet_gemm on the COMET step's dominant shapes, with and without the fused
epilogue, against torch.matmul (hipBLASLt) on the same operands, random data.

    python tools/gemm_bench.py > gpurun_out/gemm_bench.txt
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

SHAPES = [  # (M, N, K, act, out dtype, resid)
    (74368, 3072, 768, 1, torch.bfloat16, False),
    (74368, 3072, 768, 0, torch.bfloat16, False),
    (74368, 768, 3072, 0, torch.float32, True),
    (74368, 2304, 768, 0, torch.bfloat16, False),
    (73728, 1536, 384, 1, torch.bfloat16, False),
    (73728, 1536, 384, 0, torch.bfloat16, False),
    (73728, 1152, 384, 0, torch.bfloat16, False),
    (73728, 384, 1536, 0, torch.float32, True),
    (65536, 1024, 256, 1, torch.bfloat16, False),
    (73728, 384, 384, 0, torch.float32, True),
    (65536, 384, 1536, 0, torch.float32, True),
    (65536, 256, 1024, 0, torch.float32, True),
    (65536, 768, 384, 0, torch.bfloat16, False),
    (8192, 384, 1536, 0, torch.float32, True),
    (8192, 384, 384, 0, torch.float32, True),
    (8192, 1536, 384, 1, torch.bfloat16, False),
    (8192, 1152, 384, 0, torch.bfloat16, False),
    (74368, 768, 768, 0, torch.float32, True),
    (8192, 8192, 8192, 0, torch.bfloat16, False),
]


def bench(fn, iters=20):
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
    dev = "cuda"
    print(f"{'M':>6} {'N':>5} {'K':>5} act out res | comet ms  TF/s | torch ms TF/s | ratio")
    for M, N, K, act, odt, res in SHAPES:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) * 0.05
        b = torch.rand(N, device=dev)
        r = torch.rand(M, N, device=dev, dtype=odt) if res else None
        out = torch.empty(M, N, device=dev, dtype=odt)
        os.environ["COMET_GEMM_NO_SK"] = "1"
        t_pp = bench(lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt))
        os.environ["COMET_GEMM_NO_PP"] = "1"
        t_old = bench(lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt))
        ref_out = out.clone()
        del os.environ["COMET_GEMM_NO_PP"]
        del os.environ["COMET_GEMM_NO_SK"]
        t = bench(lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt))
        err = (out.float() - ref_out.float()).abs().max().item()
        extra = ""
        if os.environ.get("COMET_GEMM_AB"):  # A/B switch named by COMET_GEMM_AB (e.g. COMET_GEMM_NO_WIDE)
            os.environ[os.environ["COMET_GEMM_AB"]] = "1"
            tb = bench(lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt))
            del os.environ[os.environ["COMET_GEMM_AB"]]
            extra = f" | {os.environ['COMET_GEMM_AB']} {fl_ / tb / 1e9 if (fl_ := 2.0 * M * N * K) else 0:6.0f} TF/s"
        tt = bench(lambda: torch.matmul(x, w.t()))
        fl = 2.0 * M * N * K
        print(f"{M:6d} {N:5d} {K:5d} {act:3d} {str(odt)[6:]:>4} {int(res):3d} | {t:8.3f} {fl / t / 1e9:6.0f} | "
              f"{tt:8.3f} {fl / tt / 1e9:5.0f} | {tt / t:5.2f} | no-SK {fl / t_pp / 1e9:6.0f} | 256-row {fl / t_old / 1e9:6.0f} TF/s, "
              f"max|new-old| {err:.2e}{extra}", flush=True)


if __name__ == "__main__":
    main()
