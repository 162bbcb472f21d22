#!/bin/bash
# Round 5: op-level determinism under HBM noise (tools/race_stress.py) on the default library.
#   bash tools/gpu/r05m.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u tools/race_stress.py ${REPS:-200} > $O/race.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/race.txt; echo "race rc $rc"
