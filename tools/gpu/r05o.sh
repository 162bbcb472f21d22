#!/bin/bash
# Round 5: first differing kernel output between repeated forwards, one process alone and two
# processes sharing the GPU (tools/op_trace_det.py).
#   bash tools/gpu/r05o.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/op_trace_det.py > $O/solo.txt 2>&1 || { echo "solo failed"; tail $O/solo.txt; exit 1; }
grep pass $O/solo.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/op_trace_det.py > $O/pair${r}_a.txt 2>&1 &
  pa=$!
  timeout -k 10 300 python -u tools/op_trace_det.py > $O/pair${r}_b.txt 2>&1
  rb=$?; wait $pa; ra=$?
  echo "== pair $r rc $ra $rb"; grep -h -A1 pass $O/pair${r}_a.txt $O/pair${r}_b.txt
  [ $ra -eq 0 ] && [ $rb -eq 0 ] || exit 1
done
echo done
