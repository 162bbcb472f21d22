#!/bin/bash
# Three separate rocprofv3 counter passes over a short bench run (kernel-trace only alongside the
# counters), summarised per kernel instance into profiles/<tag>_pmc.json by tools/pmc_summary.py.
#   bash tools/gpu/pmc.sh <tag>
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
B="python bench.py --no-cpu-baseline --steps 1 --warmup 1"
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_mfma -o run -- $B > $O/pmc_mfma.log 2>&1 || { echo "mfma pass failed $?"; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_fetch -o run -- $B > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed $?"; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_write -o run -- $B > $O/pmc_write.log 2>&1 || { echo "write pass failed $?"; exit 1; }
python tools/pmc_summary.py --config '{"batch": 8, "frames": 16, "image": 512, "tracks": 512}' --out $O/$(basename $TAG)_pmc.json $O/pmc_mfma $O/pmc_fetch $O/pmc_write > $O/pmc_summary.txt 2>&1 || { tail $O/pmc_summary.txt; exit 1; }
head -40 $O/pmc_summary.txt
