#!/bin/bash
# Round 5: row-LN tile height for the M = 65536 shapes: default (128 x 384 at K >= 1024, 64 x 384
# below), COMET_ROWLN_HALF=1 (64 x 384 everywhere), COMET_ROWLN_32ALL=1 (32 x 384 for every
# N = 384 shape) -- rowln_lib_ab.py A/B/C/A/B/C, row-LN op tests for the 32-row arm, bench step.
#   bash tools/gpu/r05q.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
env COMET_ROWLN_32ALL=1 timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k rowln > $O/tests_32all.log 2>&1
rc=$?; tail -2 $O/tests_32all.log; [ $rc -le 1 ] || exit 1
for r in 1 2; do
  step timeout -k 10 200 python -u tools/rowln_lib_ab.py default > $O/rowln_default.$r.txt 2>&1
  step env COMET_ROWLN_HALF=1 timeout -k 10 200 python -u tools/rowln_lib_ab.py half > $O/rowln_half.$r.txt 2>&1
  step env COMET_ROWLN_32ALL=1 timeout -k 10 200 python -u tools/rowln_lib_ab.py r32 > $O/rowln_r32.$r.txt 2>&1
done
paste -d'\n' $O/rowln_default.1.txt $O/rowln_half.1.txt $O/rowln_r32.1.txt | grep -v amdgpu.ids
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  for arm in default HALF 32ALL; do
    if [ $arm = default ]; then step timeout -k 10 300 $B > $O/bench_$arm.$r.json 2> $O/bench_$arm.$r.err
    else step env COMET_ROWLN_$arm=1 timeout -k 10 300 $B > $O/bench_$arm.$r.json 2> $O/bench_$arm.$r.err; fi
    python -c "import json; d=json.loads(open('$O/bench_$arm.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$arm $r', d['value'], d['ms_per_step'], k['comet_gemm_rowln']['ms_per_step'])"
  done
done
echo done
