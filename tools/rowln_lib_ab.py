"""comet_gemm_rowln timing on the tracker's row-LN shapes for one library build (COMET_HIP_LIB):
run it once per build, alternating builds, and compare the lines (tools/gpu/rowln_ab.sh).

    COMET_HIP_LIB=... python tools/rowln_lib_ab.py [tag]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

SHAPES = [  # (M, N, K, raw, y16, z16): the step's rowln calls (profiles/r03_v3/gemm_shapes.txt)
    (65536, 384, 384, True, True, False), (65536, 384, 1536, False, True, True), (65536, 384, 1536, False, True, False),
    (8192, 384, 1536, False, True, False), (8192, 384, 384, True, True, False), (65536, 256, 1024, False, True, False),
    (65536, 256, 256, True, True, False), (8192, 384, 1536, False, True, True),
]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("COMET_HIP_LIB", "default")
    dev = "cuda"
    for M, N, K, raw, y16, z16 in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.rand(N, device=dev, generator=g)
        r = torch.rand(M, N, device=dev, generator=g)
        z = (torch.ones(N, device=dev), torch.zeros(N, device=dev), 1e-5) if z16 else None

        def run():
            return ops.linear_rowln(x, w, b, r, raw=raw, y16_eps=1e-6 if y16 else None, z=z)
        out = run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        c = out[0].float()
        ck = float(c.double().sum())
        print(f"{M:6d} {N:4d} {K:5d} raw{int(raw)} y{int(y16)} z{int(z16)}: {min(ts) * 1e3:8.1f} us  checksum {ck:.6e}  [{tag}]",
              flush=True)


if __name__ == "__main__":
    main()
