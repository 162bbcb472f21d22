#!/bin/bash
# SQ counter pass over single persistent-GEMM shapes (tools/gemm_one.py), one rocprofv3 --pmc run
# per shape and counter set (<= 8 SQ counters, no trace domains), summarised by tools/pmc_summary.py.
#   bash tools/gpu/gemm_pmc.sh <tag>      -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
i=0
for shape in "73728 1536 384 1 bf16 0" "74368 3072 768 1 bf16 0" "74368 768 768 0 f32 1" "65536 384 1536 0 f32 1"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --kernel-trace -f csv -d $O/s$i -o run -- python tools/gemm_one.py $shape 10 > $O/s$i.log 2>&1 || { echo "pass $i failed $?"; exit 1; }
  tail -1 $O/s$i.log
done
python - $O <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for d in sorted(glob.glob(os.path.join(O, "s*"))):
    if not os.path.isdir(d):
        continue
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        if "gemm" not in r.get("Kernel_Name", ""):
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    n = max((len(v) for v in agg.values()), default=0)
    print(os.path.basename(d), {k: round(sum(v) / max(len(v), 1)) for k, v in sorted(agg.items())}, "dispatch-rows", n)
PY
