"""LayerNorm backward (comet_layernorm_bwd / _res) on the camera head's shapes, per rows-per-wave
setting (COMET_LNB_RPW): HIP-event time and effective HBM rate.

    python tools/lnbwd_bench.py
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
    torch.manual_seed(0)
    for rows, mode in [(69240, "dual"), (69240, "res"), (73856, "res"), (65536, "affine")]:
        C = 768
        x = torch.randn(rows, C, device="cuda")
        dy = torch.randn(rows, C, device="cuda")
        dy2 = torch.randn(rows, C, device="cuda").to(torch.bfloat16)
        dres = torch.randn(rows, C, device="cuda")
        mean, rstd = torch.randn(rows, device="cuda"), torch.rand(rows, device="cuda") + 0.5
        w = torch.rand(C, device="cuda")
        dw, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        if mode == "dual":
            fn = lambda: ops.layernorm_bwd(x, dy, mean, rstd, dy2=dy2)
            nbytes = rows * C * (4 + 4 + 2 + 4)
        elif mode == "res":
            fn = lambda: ops.layernorm_bwd_res(x, dy, dres, mean, rstd)
            nbytes = rows * C * (4 + 4 + 4 + 4)
        else:
            fn = lambda: ops.layernorm_bwd(x, dy, mean, rstd, w, dw, db)
            nbytes = rows * C * (4 + 4 + 4)
        ref = fn().clone()
        line = []
        for rpw in ("16", "8", "4", "2", "1"):
            os.environ["COMET_LNB_RPW"] = rpw
            us = timed(fn)
            same = torch.equal(fn(), ref)
            line.append(f"rpw {rpw}: {us:6.1f} us {nbytes / us / 1e6:5.2f} TB/s{'' if same else ' DIFF'}")
        os.environ.pop("COMET_LNB_RPW")
        print(f"rows {rows} {mode:6s}: " + " | ".join(line), flush=True)


if __name__ == "__main__":
    main()
