#!/bin/bash
# One GPU call for the round's open measurements, each step under its own time limit, stopping at
# the first failure: the rows of the opt-in features' tests, their A/B against the defaults (row-LN
# tile micro-benchmark, whole bench step with / without COMET_MLP_FUSE=1 and COMET_ROWLN_32=1). The
# measurement pass (tools/gpu/measure.sh) and the PMC passes (tools/gpu/pmc.sh) are calls of their own.
#   bash tools/gpu/round4.sh <tag>   -> gpurun_out/<tag>*/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "dact or mlp_fused or rowln or corr" > $O/tests_new.log 2>&1
tail -2 $O/tests_new.log
step timeout -k 10 100 python -u tools/rowln_lib_ab.py default > $O/rowln32_ab.txt 2>&1
step env COMET_ROWLN_32=1 timeout -k 10 100 python -u tools/rowln_lib_ab.py rowln32 >> $O/rowln32_ab.txt 2>&1
step timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_default.json 2> $O/bench_default.err
step env COMET_MLP_FUSE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_mlpfuse.json 2> $O/bench_mlpfuse.err
step env COMET_ROWLN_32=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_rowln32.json 2> $O/bench_rowln32.err
for f in bench_default bench_mlpfuse bench_rowln32; do
  python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"
done
echo done
