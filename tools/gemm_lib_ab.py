"""comet_gemm timing on the step's persistent-GEMM shapes for one library build (COMET_HIP_LIB), with a
correctness check against torch (bf16 operands, f32 math): run it once per build, alternating builds
(A/B/A/B), and compare the lines.

    COMET_HIP_LIB=... python tools/gemm_lib_ab.py [tag]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import _lib as L, ops  # noqa: E402

SHAPES = [  # (M, N, K, act, out dtype, resid, aux)
    (65536, 1536, 384, 1, torch.bfloat16, False, False),
    (74368, 3072, 768, 1, torch.bfloat16, False, False),
    (74368, 2304, 768, 0, torch.bfloat16, False, False),
    (65536, 1152, 384, 0, torch.bfloat16, False, False),
    (65536, 1024, 256, 1, torch.bfloat16, False, False),
    (65536, 768, 384, 0, torch.bfloat16, False, False),
    (73856, 3072, 768, 1, torch.bfloat16, False, True),
    (74368, 768, 3072, 0, torch.float32, True, False),
    (8192, 8192, 8192, 0, torch.bfloat16, False, False),
    # the virtual-track shapes (M = 8192: 128 x 384 / 64 x 384 / 128 x 256 tiles)
    (8192, 1536, 384, 1, torch.bfloat16, False, False),
    (8192, 1152, 384, 0, torch.bfloat16, False, False),
    (8192, 768, 384, 0, torch.bfloat16, False, False),
    (8192, 384, 384, 0, torch.bfloat16, False, False),
    (8192, 384, 1536, 0, torch.float32, True, False),
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
    tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(L.LIB_PATH)
    torch.manual_seed(0)
    for M, N, K, act, odt, res, aux in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.rand(N, device="cuda")
        r = torch.rand(M, N, device="cuda", dtype=odt) if res else None
        out = torch.empty(M, N, device="cuda", dtype=odt)
        ax = torch.empty(M, N, device="cuda", dtype=odt) if aux else None
        fn = lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt, aux=ax)  # noqa: E731
        t = bench(fn)
        rows = slice(0, 4096)
        pre = x[rows].float() @ w.float().t() + b
        ref = torch.nn.functional.gelu(pre) if act == 1 else pre
        if res:
            ref = ref + r[rows].float()
        err = ((out[rows].float() - ref).abs() / (ref.abs() + 1e-2)).max().item()
        aerr = ((ax[rows].float() - pre).abs() / (pre.abs() + 1e-2)).max().item() if aux else 0.0
        ok = err < 1.6e-2 and aerr < 1.6e-2
        print(f"{tag} M{M} N{N} K{K} act{act} {str(odt)[6:]} res{int(res)} aux{int(aux)}: {t * 1e3:8.1f} us "
              f"{2 * M * N * K / t / 1e9:6.0f} TF/s  rel err {err:.1e} aux {aerr:.1e} {'ok' if ok else 'BAD'}", flush=True)


if __name__ == "__main__":
    main()
