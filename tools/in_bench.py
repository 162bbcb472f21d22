"""InstanceNorm (comet_instnorm_nhwc) on the fine ShallowEncoder's small-image shapes: the
one-wave-per-image kernel vs the one-block-per-image kernel (COMET_IN_NO_WAVE=1).

    python tools/in_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from comet_amd import ops  # noqa: E402
from tile_bench import timed  # noqa: E402


def main():
    for n, h, w, c, resid in [(65536, 16, 16, 32, False), (65536, 8, 8, 32, True), (65536, 8, 8, 32, False),
                              (65536, 4, 4, 32, True)]:
        x = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16)
        r = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16) if resid else None
        fn = lambda: ops.instnorm_nhwc(x, r, relu=True, relu_inner=resid)
        nbytes = x.numel() * 2 * (3 if resid else 2)
        t_wave = timed(fn)
        yw = fn().clone()
        os.environ["COMET_IN_NO_WAVE"] = "1"
        t_blk = timed(fn)
        yb = fn()
        os.environ.pop("COMET_IN_NO_WAVE")
        d = (yw.float() - yb.float()).abs().max().item()
        print(f"[{n},{h},{w},{c}] res={resid}: wave {t_wave:7.1f} us ({nbytes / t_wave / 1e6:4.2f} TB/s)  "
              f"block {t_blk:7.1f} us ({nbytes / t_blk / 1e6:4.2f} TB/s)  max|diff| {d:.3g}", flush=True)


if __name__ == "__main__":
    main()
