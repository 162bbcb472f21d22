"""Times comet_corr_sample at the coarse tracker's shape (B=8, S=16, N=512, 4 levels from 64^2,
C=128, r=4) and the fine one (C=32, r=3 on 31x31 patch maps), per kernel variant (env)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402


def run(C, r, B, N, S, H0, levels, reps=10):
    pyr = [torch.randn(B * S, H0 >> l, H0 >> l, C, device="cuda").to(torch.bfloat16) for l in range(levels)]
    rows = B * N * S
    feats = torch.randn(rows, C, device="cuda")
    coords = torch.rand(rows, 2, device="cuda") * (H0 - 1)
    win = 2 * r + 1
    out = torch.empty(rows, levels * win * win, device="cuda")
    res = {}
    for name, env in (("v1", None), ("pf", "1")):
        if env:
            os.environ["COMET_CORR_PF"] = env
        else:
            os.environ.pop("COMET_CORR_PF", None)
        ops.corr_sample(pyr, r, feats, coords, out, 0, B, N, S)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.corr_sample(pyr, r, feats, coords, out, 0, B, N, S)
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / reps * 1e3
        res[name + "_out"] = out.clone()
    d = (res["v1_out"] - res["pf_out"]).abs().max().item()
    print(f"C={C} r={r} rows={rows}: v1 {res['v1']:.1f} us, pf {res['pf']:.1f} us, max diff {d:.2e}", flush=True)


run(128, 4, 8, 512, 16, 64, 4)
run(32, 3, 8 * 512, 1, 15, 31, 1)
