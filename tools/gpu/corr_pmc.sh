#!/bin/bash
# Counter passes over tools/corr_one.py (the coarse correlation kernel alone): bash tools/gpu/corr_pmc.sh <tag>
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
P="python tools/corr_one.py 5"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $P > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --kernel-trace -f csv -d $O/sq -o run -- $P > $O/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d $O/sq2 -o run -- $P > $O/sq2.log 2>&1 || { echo "sq2 pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo done
