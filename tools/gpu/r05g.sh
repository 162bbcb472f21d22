#!/bin/bash
# Round 5: run-to-run determinism of the training step (tools/determinism.py) on the default
# library and with single paths switched off, then the GEMM k-loop counters (r05f.sh).
#   bash tools/gpu/r05g.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
for arm in DEFAULT COMET_ROWLN_NOSPLIT COMET_MLP_UNFUSE COMET_TOKENS_ROWS COMET_CORR_VALU COMET_ROWLN_NO32; do
  if [ $arm = DEFAULT ]; then
    step timeout -k 10 200 python -u tools/determinism.py 1 bf16 > $O/det_$arm.txt 2>&1
  else
    step env $arm=1 timeout -k 10 200 python -u tools/determinism.py 1 bf16 > $O/det_$arm.txt 2>&1
  fi
  echo "== $arm"; head -12 $O/det_$arm.txt | grep -v amdgpu.ids
done
step bash tools/gpu/r05f.sh $TAG/pmc
echo done
