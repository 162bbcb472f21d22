"""The fine ShallowEncoder's last up-sampling (65536 patches, 16 x 16 -> 31 x 31 x 32 bf16) with the
fine pyramid's 2 x 2 average pool: separate kernels (resize, then avgpool2) against the fused
comet_resize_bilinear_pool_nhwc, HIP events.

    python tools/resize_pool_bench.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "comet-pose-estimation_amd")]
from comet_amd import ops  # noqa: E402
from tile_bench import timed  # noqa: E402


def main():
    x = torch.randn(65536, 16, 16, 32, device="cuda").to(torch.bfloat16)
    w = (torch.randn(32, 32, device="cuda") * 0.2).to(torch.bfloat16)
    b = torch.randn(32, device="cuda")
    conv = lambda: ops.linear(x.reshape(-1, 32), w, bias=b, resid=x.reshape(-1, 32), out_dtype=torch.bfloat16)  # noqa: E731
    sep = lambda: ops.avgpool2_nhwc(ops.resize_bilinear(x, 31, 31, nhwc=True))  # noqa: E731
    fused = lambda: ops.resize_bilinear_pool(x, 31, 31)  # noqa: E731
    tail = lambda: ops.conv1x1_resize_pool(x, w, b, 31, 31)  # noqa: E731
    nbytes = x.numel() * 2 + 65536 * (31 * 31 + 15 * 15) * 32 * 2
    for rep in range(2):
        c, a, f, t = timed(conv), timed(sep), timed(fused), timed(tail)
        print(f"conv2 GEMM {c:7.1f} us + resize, avgpool2 {a:7.1f} us | + resize_pool {f:7.1f} us "
              f"({nbytes / f / 1e6:.2f} TB/s) | conv1x1_resize_pool {t:7.1f} us ({nbytes / t / 1e6:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
