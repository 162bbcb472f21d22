#!/bin/bash
# Counter passes (one rocprofv3 run each, kernel-trace only beside the counters) over a short GPU
# program: bash tools/gpu/prog_pmc.sh <tag> <python script> [args...]; summarise with
# python tools/pmc_kernel.py gpurun_out/<tag> <kernel regex>
set -o pipefail
TAG=${1:?tag}; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python "$@" > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --kernel-trace -f csv -d $O/sq -o run -- python "$@" > $O/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR --kernel-trace -f csv -d $O/sq2 -o run -- python "$@" > $O/sq2.log 2>&1 || { echo "sq2 pass failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/fetch -o run -- python "$@" > $O/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
echo done
