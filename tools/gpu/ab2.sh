#!/bin/bash
# A/B/A of two env switches on the bench line (same box): bash tools/gpu/ab2.sh <tag> <ENV=V> <ENV=V>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$1
mkdir -p $O
run() { env $2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/$1.json 2> $O/$1.err || exit 1; python -c "import json;d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]);print('$1 $2',d['value'],d['ms_per_step'])"; }
run new X=1
run off1 "$2"
run off2 "$3"
run new2 X=1
