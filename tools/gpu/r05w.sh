#!/bin/bash
# Round 5 final tree (suite: r05v): smoke(), the default bench line (CPU baseline leg on)
# and the kernel-trace statistics of the bench step.
#   bash tools/gpu/r05w.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/smoke.log
step timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
tail -c 400 $O/bench.json
step timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err
echo done
