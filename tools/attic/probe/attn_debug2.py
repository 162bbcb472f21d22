import sys, torch
sys.path.insert(0, "comet-pose-estimation_amd")
from comet_amd import ops
B, H, D, L = 1, 1, 32, 64
q = torch.zeros(B, 16, D).bfloat16().cuda(); k = torch.zeros(B, L, D).bfloat16().cuda()
for K0 in range(L):
    v = torch.zeros(B, L, D); v[0, K0, K0 % 32] = 64.0
    o = ops.attention(q, k, v.bfloat16().cuda(), H).float().cpu()[0]
    nz = (o.abs() > 1e-3).nonzero().tolist()
    rows = sorted(set(r for r, c in nz)); cols = sorted(set(c for r, c in nz))
    print(K0, "expect col", K0 % 32, "got cols", cols, "vals", [round(o[0, c].item(), 3) for c in cols], "rows", len(rows))
