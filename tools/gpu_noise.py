"""GPU load from another process for concurrency experiments: torch (hipBLASLt) GEMMs and HBM copies
for SECONDS, none of this library's kernels.

    python tools/gpu_noise.py [seconds]
"""
import sys
import time

import torch

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
x = torch.empty(256 * 2**20, device="cuda")
y = torch.empty_like(x)
t0 = time.time()
n = 0
while time.time() - t0 < secs:
    for _ in range(4):
        c = a @ b
        y.copy_(x)
    torch.cuda.synchronize()
    n += 1
print(f"noise: {n} rounds in {time.time() - t0:.1f} s", flush=True)
