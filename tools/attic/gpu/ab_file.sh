#!/bin/bash
# A/B of a Python source change on the bench line, on one box:
#   bash tools/gpu/ab_file.sh <tag> <repo file> <old copy>
# runs new, old (old copy swapped in), new again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$1
mkdir -p $O
cp $2 $O/new_src.py
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/a.json 2> $O/a.err || exit 1
cp $3 $2
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b.json 2> $O/b.err; rc=$?
cp $O/new_src.py $2
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/a2.json 2> $O/a2.err || exit 1
for f in a b a2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'])"; done
