#!/bin/bash
# Round 5: op-level determinism under HBM noise (tools/race_stress.py), then the persistent-GEMM
# intra-k-tile stamps (r05k.sh).
#   bash tools/gpu/r05l.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u tools/race_stress.py 30 > $O/race.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/race.txt; echo "race rc $rc"
[ $rc -eq 0 ] || exit 1
bash tools/gpu/r05k.sh $TAG/stamps || exit 1
echo done
