#!/bin/bash
# Persistent-GEMM phase stamps (default vs park-all probe build) and HBM traffic per launch
#   bash tools/gpu/stamp_ab.sh <tag>
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for lib in stamp stamp_park; do
  for sh in "73728 1536 384 1 bf16 0" "73728 1536 384 0 bf16 0" "74368 3072 768 1 bf16 0" "74368 2304 768 0 bf16 0"; do
    COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_$lib.so timeout -k 10 60 python -u tools/gemm_stamps.py $sh >> $O/stamps_$lib.txt 2>&1 || { echo "stamps failed $lib $sh"; tail $O/stamps_$lib.txt; exit 1; }
  done
done
for lib in stamp stamp_park; do
  for c in FETCH_SIZE WRITE_SIZE; do
    COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_$lib.so timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -f csv -d $O/pmc_${lib}_$c -o run -- python tools/gemm_one.py 73728 1536 384 1 bf16 0 10 > $O/pmc_${lib}_$c.log 2>&1 || { echo "pmc failed $lib $c"; exit 1; }
  done
done
python - $O <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for d in sorted(glob.glob(os.path.join(O, "pmc_*"))):
    if not os.path.isdir(d):
        continue
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_w4" in r.get("Kernel_Name", ""):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(os.path.basename(d), {k: f"{sum(v) / len(v) / 1e6:.1f} MB/launch (n={len(v)})" for k, v in vals.items()})
PY
cat $O/stamps_stamp.txt $O/stamps_stamp_park.txt | grep -v amdgpu.ids
