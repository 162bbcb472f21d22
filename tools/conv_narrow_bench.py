"""comet_conv2d_nhwc narrow-output path (cout <= 64, short K) on the fine ShallowEncoder's shapes
(65536 patches, blocks.py ShallowEncoder; refine_track.py:62-120), bf16 in / out, for one library
build (COMET_HIP_LIB): run once per build, alternating builds, and compare the lines.

    COMET_HIP_LIB=... python tools/conv_narrow_bench.py [tag]
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from comet_amd import _lib as L, ops  # noqa: E402
from tile_bench import timed  # noqa: E402

SHAPES = [  # (n, h, w, c, cout, k, stride, pad)
    (65536, 31, 31, 8, 32, 3, 2, 1), (65536, 16, 16, 32, 32, 3, 2, 1), (65536, 8, 8, 32, 32, 3, 1, 1),
    (65536, 16, 16, 32, 32, 1, 2, 0), (65536, 8, 8, 32, 32, 3, 2, 1), (65536, 4, 4, 32, 32, 3, 1, 1),
    # the BasicEncoder's 7x7 stride-2 stem (3 channels padded to 8, frames halved to 256^2)
    (128, 256, 256, 8, 64, 7, 2, 3),
]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(L.LIB_PATH)
    torch.manual_seed(0)
    for n, h, w, c, cout, k, s, p in SHAPES:
        x = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16)
        K = c * k * k
        wm = (torch.randn(cout, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
        b = torch.randn(cout, device="cuda")
        fn = lambda: ops.conv2d_nhwc(x, wm, k, k, s, p, bias=b, out_dtype=torch.bfloat16)  # noqa: E731
        t = timed(fn)
        y = fn()
        oh, ow = y.shape[1], y.shape[2]
        ref = torch.nn.functional.conv2d(x[:64].permute(0, 3, 1, 2).float().cpu(),
                                         wm.float().cpu().reshape(cout, k, k, c).permute(0, 3, 1, 2), b.cpu(),
                                         stride=s, padding=p).permute(0, 2, 3, 1)
        err = (y[:64].float().cpu() - ref).abs().max().item()
        byts = x.numel() * 2 + y.numel() * 2
        print(f"{tag} conv {k}x{k}s{s} c{c}->{cout} {h}x{w} n{n}: {t:8.1f} us  {byts / t / 1e3:6.0f} GB/s  "
              f"max err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
