"""Times comet_corr_sample at the coarse tracker's shape (B=8, S=16, N=512, 4 levels from 64^2,
C=128, r=4) and the fine one (C=32, r=3 on 31x31 patch maps) for each dispatch variant: the
matrix-core kernel at 4 waves per SIMD (default), at 3 (COMET_CORR_OCC3=1) and with a 3 / 4-deep
pixel ring (COMET_CORR_RING, 3 waves per SIMD), and the VALU kernel (COMET_CORR_VALU=1); max
difference against the first variant.

    python tools/corr_bench.py > gpurun_out/corr_bench.txt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

VARIANTS = [("mfma occ4", {}), ("mfma occ3", {"COMET_CORR_OCC3": "1"}), ("mfma ring3", {"COMET_CORR_RING": "3"}),
            ("mfma ring4", {"COMET_CORR_RING": "4"}), ("valu", {"COMET_CORR_VALU": "1"})]


def run(C, r, B, N, S, H0, levels, reps=10, clustered=False):
    pyr = [torch.randn(B * S, H0 >> l, H0 >> l, C, device="cuda").to(torch.bfloat16) for l in range(levels)]
    rows = B * N * S
    feats = torch.randn(rows, C, device="cuda")
    coords = torch.rand(rows, 2, device="cuda") * (H0 - 1)
    if clustered:  # tracks in a few clumps (keypoints on textured objects)
        centers = torch.rand(B * S * 8, 2, device="cuda") * (H0 - 1)
        idx = torch.randint(0, 8, (rows,), device="cuda") + (torch.arange(rows, device="cuda") % S) * 8
        coords = (centers[idx] + torch.randn(rows, 2, device="cuda") * 3).clamp(0, H0 - 1)
    win = 2 * r + 1
    out = torch.empty(rows, levels * win * win, device="cuda")
    first = None
    for name, env in VARIANTS:
        for k in ("COMET_CORR_RING", "COMET_CORR_VALU", "COMET_CORR_OCC3"):
            os.environ.pop(k, None)
        os.environ.update(env)
        ops.corr_sample(pyr, r, feats, coords, out, 0, B, N, S)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.corr_sample(pyr, r, feats, coords, out, 0, B, N, S)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / reps * 1e3)
        if first is None:
            first = out.clone()
        d = (out - first).abs().max().item()
        print(f"C={C} r={r} rows={rows}{' clustered' if clustered else ''} {name:11s}: {min(ts):7.1f} us  max diff {d:.2e}",
              flush=True)
    for k in ("COMET_CORR_RING", "COMET_CORR_VALU", "COMET_CORR_OCC3"):
        os.environ.pop(k, None)


run(128, 4, 8, 512, 16, 64, 4)
run(128, 4, 8, 512, 16, 64, 4, clustered=True)
run(32, 3, 8 * 512, 1, 15, 31, 3)
