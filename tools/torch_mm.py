"""torch.matmul (hipBLASLt) on the step's dominant Linear shapes, for kernel-name / timing reference."""
import torch

SHAPES = [(74368, 3072, 768), (65536, 1024, 256), (73728, 1536, 384), (74368, 768, 3072)]
for M, N, K in SHAPES:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    for _ in range(5):
        torch.nn.functional.linear(x, w)
    torch.cuda.synchronize()
