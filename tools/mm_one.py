"""torch.matmul (hipBLASLt) on one shape, repeated (counter-pass companion of gemm_one.py)."""
import sys
import torch
M, N, K = (int(v) for v in sys.argv[1:4])
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
for _ in range(10):
    torch.nn.functional.linear(x, w)
torch.cuda.synchronize()
