#!/bin/bash
# Round 5: counters of the persistent GEMM's k-loop on a k-loop-bound shape (M 74368 N 2304 K 3072)
# and on the GELU K 384 shape, over tools/gemm_one.py (prog_pmc.sh passes).
#   bash tools/gpu/r05f.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step bash tools/gpu/prog_pmc.sh $TAG/k3072 tools/gemm_one.py 74368 2304 3072 0 bf16 0 20
step bash tools/gpu/prog_pmc.sh $TAG/gelu384 tools/gemm_one.py 65536 1536 384 1 bf16 0 20
python tools/pmc_kernel.py $O/k3072 gemm_w4 > $O/k3072.txt 2>&1
python tools/pmc_kernel.py $O/gelu384 gemm_w4 > $O/gelu384.txt 2>&1
cat $O/k3072.txt $O/gelu384.txt
echo done
