#!/bin/bash
# Full GPU test suite (one pytest process), then the measurement pass (tools/gpu/measure.sh).
#   bash tools/gpu/full.sh <tag>        -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/measure.sh $TAG
