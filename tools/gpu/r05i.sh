#!/bin/bash
# Round 5: determinism with two processes sharing the GPU (tools/determinism.py twice at once),
# default library and with single kernel families switched to their alternatives.
#   bash tools/gpu/r05i.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
pair() {  # $1 = arm name, rest = env assignments
  local arm=$1; shift
  env "$@" timeout -k 10 200 python -u tools/determinism.py 1 bf16 > $O/${arm}_a.txt 2>&1 &
  local pa=$!
  env "$@" timeout -k 10 200 python -u tools/determinism.py 1 bf16 > $O/${arm}_b.txt 2>&1
  local rb=$?
  wait $pa; local ra=$?
  echo "== $arm rc $ra $rb"
  grep -h "keys differ" $O/${arm}_a.txt $O/${arm}_b.txt
  grep -h "out\." $O/${arm}_a.txt | head -5
  [ $ra -eq 0 ] && [ $rb -eq 0 ] || { echo "arm $arm failed"; exit 1; }
}
ARMS=${ARMS:-default}
for arm in $ARMS; do
  case $arm in
    default) pair default X=1 ;;
    nopp) pair nopp COMET_GEMM_NO_PP=1 ;;
    attn16) pair attn16 COMET_ATTN_FWD16=1 COMET_ATTN_BWD16=1 ;;
    fwd16) pair fwd16 COMET_ATTN_FWD16=1 ;;
    bwd16) pair bwd16 COMET_ATTN_BWD16=1 ;;
    nobpark) pair nobpark COMET_GEMM_NO_BPARK=1 ;;
    nowide) pair nowide COMET_GEMM_NO_WIDE=1 ;;
    nopp384) pair nopp384 COMET_GEMM_NO_PP384=1 COMET_PP_NO_384=1 ;;
    rowlnsplit) pair rowlnsplit COMET_ROWLN_NOSPLIT=1 COMET_ROWLN_NO32=1 ;;
    prio) pair prio COMET_GEMM_PRIO=1 ;;
    pp256) pair pp256 COMET_PP_TILE=256x256 ;;
    corr_valu) pair corr_valu COMET_CORR_VALU=1 ;;
    *) echo "unknown arm $arm"; exit 1 ;;
  esac
done
echo done
