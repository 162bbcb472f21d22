#!/bin/bash
# A/B/A/B of two library builds on the persistent-GEMM shapes: bash tools/gpu/lib_ab.sh <tag> <libA> <libB>
set -o pipefail
TAG=${1:?tag}; A=${2:?libA}; B=${3:?libB}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for lib in $A $B; do
    COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 120 python -u tools/gemm_lib_ab.py $lib >> $O/lib_ab.txt 2>&1 || { echo "failed $lib"; tail $O/lib_ab.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/lib_ab.txt | sort -t: -k1,1 -s | sort -k2,2 -s
