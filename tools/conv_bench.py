"""comet_conv2d_nhwc on the BasicEncoder's 64 -> 64 shapes: the rows-in-LDS 3x3 kernel (default)
vs the implicit-GEMM 128 x 64 tile (COMET_CONV_NO_ROWS=1).

    python tools/conv_bench.py
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from comet_amd import ops  # noqa: E402
from tile_bench import timed  # noqa: E402


def main():
    for n, h, w, c, cout in [(128, 128, 128, 64, 64), (128, 64, 64, 64, 64)]:
        x = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16)
        wm = (torch.randn(cout, 9 * c, device="cuda") / math.sqrt(9 * c)).to(torch.bfloat16)
        b = torch.randn(cout, device="cuda")
        fn = lambda: ops.conv2d_nhwc(x, wm, 3, 3, 1, 1, bias=b, act=2, out_dtype=torch.bfloat16)
        flop = 2.0 * n * h * w * cout * 9 * c
        t64 = timed(fn)
        y64 = fn().clone()
        os.environ["COMET_CONV_NO_ROWS"] = "1"
        t128 = timed(fn)
        y128 = fn()
        os.environ.pop("COMET_CONV_NO_ROWS")
        d = (y64.float() - y128.float()).abs().max().item()
        print(f"[{n},{h},{w},{c}]->{cout}: rows {t64:7.1f} us ({flop / t64 / 1e6:5.1f} TF/s)  "
              f"implicit GEMM {t128:7.1f} us ({flop / t128 / 1e6:5.1f} TF/s)  max diff {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
