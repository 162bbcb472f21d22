#!/bin/bash
# Round 5, fifth call: the restored tree end to end -- the whole GPU suite, the measurement pass
# (bench line with the CPU baseline, configs[1], configs[4], kernel-trace stats of the bench) and
# the three PMC passes whose summary becomes profiles/r05_pmc.json (roofline.traffic source).
#   bash tools/gpu/r05e.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"
[ $rc -le 1 ] || { echo "GPU suite ended abnormally ($rc): stopping"; exit 1; }  # 1 = test failures only
tail -2 $O/gpu_tests.log
step bash tools/gpu/measure.sh $TAG/m
step bash tools/gpu/pmc.sh $TAG/pmc
echo done
