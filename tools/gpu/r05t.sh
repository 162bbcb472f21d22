#!/bin/bash
# Round 5: the widened ping-pong default (bf16 outputs, no residual / activation / aux, K >= 768)
# against the lock-step loop everywhere (COMET_GEMM_PING=0): bench step A/B/A/B/A/B.
#   bash tools/gpu/r05t.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2 3; do
  step env COMET_GEMM_PING=0 timeout -k 10 300 $B > $O/bench_lock.$r.json 2> $O/bench_lock.$r.err
  step timeout -k 10 300 $B > $O/bench_ping.$r.json 2> $O/bench_ping.$r.err
  for arm in lock ping; do
    python -c "import json; d=json.loads(open('$O/bench_$arm.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$arm $r', d['value'], d['ms_per_step'], k['comet_gemm']['ms_per_step'])"
  done
done
echo done
