"""Persistent GEMM tile order A/B: default XCD-banded waves against per-XCD contiguous tile ranges
(COMET_GEMM_RASTER=1, read per launch), on the step's plain-GEMM shapes (tools/tile_bench.py), timed
with HIP events in alternation, with a bit-for-bit check that the order does not change the result.

    python tools/raster_ab.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "comet-pose-estimation_amd")]
from comet_amd import ops  # noqa: E402
from tile_bench import SHAPES, timed  # noqa: E402


def main():
    torch.manual_seed(0)
    for M, N, K, act, odt, res in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        b = torch.rand(N, device="cuda")
        r = torch.rand(M, N, device="cuda") if res else None
        out = torch.empty(M, N, device="cuda", dtype=odt)
        fn = lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out)
        ts, outs = {0: [], 1: []}, {}
        for rep in range(3):
            for mode in (0, 1):
                os.environ["COMET_GEMM_RASTER"] = str(mode)
                ts[mode].append(timed(fn))
                if rep == 0:
                    if r is not None:
                        r.copy_(torch.rand(M, N, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)))
                    fn()
                    outs[mode] = out.clone()
        same = torch.equal(outs[0], outs[1])
        a, c = min(ts[0]), min(ts[1])
        print(f"M {M:6d} N {N:5d} K {K:5d} act {act} {str(odt)[6:]:8s} res {int(res)}: banded {a:7.1f} us  "
              f"per-XCD {c:7.1f} us  ({(c / a - 1) * 100:+.1f} %)  identical {same}", flush=True)
        del x, w, b, r, out, outs
    os.environ.pop("COMET_GEMM_RASTER", None)


if __name__ == "__main__":
    main()
