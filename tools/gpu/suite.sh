#!/bin/bash
# Full GPU suite + smoke + the default bench line on the GPU box:
#   bash tools/gpu/suite.sh <tag>   -> gpurun_out/<tag>/{gpu_tests.log, smoke.log, bench.json}
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -15 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'cover', d.get('kernels_share_of_profiled_step'))"
