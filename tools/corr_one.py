"""A few comet_corr_sample launches at the coarse tracker's shape (B=8, S=16, N=512, 64^2 x 128
bf16, 4 levels, r=4), for rocprofv3 counter passes (tools/gpu/prog_pmc.sh <tag> tools/corr_one.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

B, N, S, H0, L, r, C = 8, 512, 16, 64, 4, 4, 128
pyr = [torch.randn(B * S, H0 >> l, H0 >> l, C, device="cuda").to(torch.bfloat16) for l in range(L)]
rows = B * N * S
feats = torch.randn(rows, C, device="cuda")
coords = torch.rand(rows, 2, device="cuda") * (H0 - 1)
out = torch.empty(rows, L * (2 * r + 1) ** 2, device="cuda")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    ops.corr_sample(pyr, r, feats, coords, out, 0, B, N, S)
torch.cuda.synchronize()
print("ok", flush=True)
