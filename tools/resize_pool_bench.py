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
    u1 = torch.randn(65536, 8, 8, 32, device="cuda").to(torch.bfloat16)
    u2 = torch.randn(65536, 4, 4, 32, device="cuda").to(torch.bfloat16)
    w = (torch.randn(32, 32, device="cuda") * 0.2).to(torch.bfloat16)
    b = torch.randn(32, device="cuda")

    def unfused():  # round 5: two resize-adds, the skinny GEMM, resize, avgpool2
        x2 = x.clone()
        ops.resize_bilinear(u1, 16, 16, nhwc=True, out=x2, add=True)
        ops.resize_bilinear(u2, 16, 16, nhwc=True, out=x2, add=True)
        t = ops.linear(x2.reshape(-1, 32), w, bias=b, resid=x2.reshape(-1, 32), out_dtype=torch.bfloat16)
        return ops.avgpool2_nhwc(ops.resize_bilinear(t.reshape(x.shape), 31, 31, nhwc=True))

    clone = lambda: x.clone()  # noqa: E731
    sep = lambda: ops.avgpool2_nhwc(ops.resize_bilinear(x, 31, 31, nhwc=True))  # noqa: E731
    fused = lambda: ops.resize_bilinear_pool(x, 31, 31)  # noqa: E731
    tail = lambda: ops.conv1x1_resize_pool(x, w, b, 31, 31, up1=u1, up2=u2)  # noqa: E731
    tail2 = lambda: ops.conv1x1_resize_pool(x, w, b, 31, 31, up1=u1, up2=u2, pool2=True)  # noqa: E731
    nbytes = (x.numel() + u1.numel() + u2.numel()) * 2 + 65536 * (31 * 31 + 15 * 15) * 32 * 2
    nbytes2 = nbytes + 65536 * 7 * 7 * 32 * 2
    for rep in range(2):
        for nt in ("0", "1"):  # COMET_RSP_NT: streaming stores of y / pool / pool2
            os.environ["COMET_RSP_NT"] = nt
            uf, cl, a, f, t, t2 = timed(unfused), timed(clone), timed(sep), timed(fused), timed(tail), timed(tail2)
            print(f"NT={nt} unfused tail {uf - cl:7.1f} us (clone excluded) | resize + avgpool2 {a:7.1f} us | "
                  f"resize_pool {f:7.1f} us | conv1x1_resize_pool with both adds {t:7.1f} us "
                  f"({nbytes / t / 1e6:.2f} TB/s algorithmic), + pool2 {t2:7.1f} us ({nbytes2 / t2 / 1e6:.2f} TB/s)",
                  flush=True)


if __name__ == "__main__":
    main()
