#!/bin/bash
# Round 5 final tree: configs[1] (fwd-only) and configs[4] (stress) bench lines, then the three PMC
# passes of the bench step (tools/gpu/pmc.sh) so roofline.traffic is from the final tree.
#   bash tools/gpu/r05u.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step timeout -k 10 300 python bench.py --no-cpu-baseline --fwd-only > $O/fwd.json 2> $O/fwd.err
tail -c 300 $O/fwd.json
step timeout -k 10 400 python bench.py --no-cpu-baseline --batch 4 --frames 64 --image 768 --steps 2 --warmup 1 > $O/stress.json 2> $O/stress.err
tail -c 300 $O/stress.json
step bash tools/gpu/pmc.sh $TAG/pmc
echo done
