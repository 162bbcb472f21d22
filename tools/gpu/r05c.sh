#!/bin/bash
# Round 5, third call: the whole GPU suite on the current tree, the per-shape census of one train
# step (tools/gemm_shapes.py) and the default bench line.
#   bash tools/gpu/r05c.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 500 --timeout-method thread tests > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step timeout -k 10 300 python -u tools/gemm_shapes.py > $O/gemm_shapes.txt 2> $O/gemm_shapes.err
step timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])"
echo done
