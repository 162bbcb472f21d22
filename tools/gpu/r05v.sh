#!/bin/bash
# Round 5: the ping-pong k-loop also for residual / f32 outputs at K >= 2048 (default) against the
# lock-step loop (COMET_GEMM_PING=0) on the step's f32 + residual K 3072 shape, A/B x 3; the GPU
# suite and two bench lines of the new default.
#   bash tools/gpu/r05v.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
for r in 1 2 3; do
  step env COMET_GEMM_PING=0 timeout -k 10 120 python tools/gemm_one.py 74368 768 3072 0 f32 1 50 >> $O/shape_lock.txt 2>&1
  step timeout -k 10 120 python tools/gemm_one.py 74368 768 3072 0 f32 1 50 >> $O/shape_default.txt 2>&1
done
grep -h "us" $O/shape_lock.txt $O/shape_default.txt
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -1 $O/gpu_tests.log
[ $rc -le 1 ] || { echo "GPU suite ended abnormally ($rc): stopping"; exit 1; }
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  step timeout -k 10 300 $B > $O/bench.$r.json 2> $O/bench.$r.err
  python -c "import json; d=json.loads(open('$O/bench.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('bench $r', d['value'], d['ms_per_step'], k['comet_gemm']['ms_per_step'])"
done
echo done
