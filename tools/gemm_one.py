"""Run one comet_gemm shape repeatedly (for rocprofv3 counter passes on a single kernel).

    python tools/gemm_one.py M N K [act] [f32|bf16] [resid] [iters] [nobias]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    act = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    odt = torch.float32 if len(sys.argv) > 5 and sys.argv[5] == "f32" else torch.bfloat16
    res = len(sys.argv) > 6 and sys.argv[6] == "1"
    iters = int(sys.argv[7]) if len(sys.argv) > 7 else 20
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = None if len(sys.argv) > 8 and sys.argv[8] == "nobias" else torch.rand(N, device="cuda")
    r = torch.rand(M, N, device="cuda", dtype=odt) if res else None
    out = torch.empty(M, N, device="cuda", dtype=odt)
    for _ in range(3):
        ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / iters
    print(f"M{M} N{N} K{K} act{act} {odt} res{int(res)}: {t * 1e3:.1f} us  {2 * M * N * K / t / 1e9:.0f} TF/s")


if __name__ == "__main__":
    main()
