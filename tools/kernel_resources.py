"""Print VGPRs / scratch / occupancy / LDS per kernel of a HIP source (hipcc remarks).
    python tools/kernel_resources.py comet-pose-estimation_amd/csrc/gemm.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", src,
                      "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        dem = k if "--mangled" in sys.argv else subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
        print(f"vgpr {v.get('VGPRs', '?'):>4} agpr {v.get('AGPRs', '?'):>3} scratch {v.get('ScratchSize', '?'):>4} "
              f"occ {v.get('Occupancy', '?')} lds {v.get('LDS Size', '?'):>6}  {dem[:150]}")
