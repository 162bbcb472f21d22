#!/bin/bash
# A/B/A/B of two library builds: bash tools/gpu/lib_ab.sh <tag> <libA> <libB> [script]
# (script: tools/gemm_lib_ab.py, the persistent-GEMM shapes, by default; tools/rowln_lib_ab.py the row-LN ones)
set -o pipefail
TAG=${1:?tag}; A=${2:?libA}; B=${3:?libB}; S=${4:-tools/gemm_lib_ab.py}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for lib in $A $B; do
    COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 120 python -u $S $lib >> $O/lib_ab.txt 2>&1 || { echo "failed $lib"; tail $O/lib_ab.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/lib_ab.txt | sort -t: -k1,1 -s | sort -k2,2 -s
