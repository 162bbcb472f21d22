#!/bin/bash
# Round 5: intra-k-tile clock stamps of the persistent GEMM (diagnostic build libcomet_hip_stamp.so,
# tools/gemm_stamps.py): where a steady k-tile's cycles go, per wave of one SIMD pair.
#   bash tools/gpu/r05k.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
L=comet-pose-estimation_amd/libcomet_hip_stamp.so
for shape in "74368 2304 3072 0 bf16 0" "74368 2304 768 0 bf16 0" "65536 1536 384 1 bf16 0" "74368 768 3072 0 f32 1" "8192 8192 8192 0 bf16 0"; do
  COMET_HIP_LIB=$L timeout -k 10 120 python -u tools/gemm_stamps.py $shape >> $O/stamps.txt 2>&1 || { echo "stamps failed: $shape"; exit 1; }
done
grep -v amdgpu.ids $O/stamps.txt
echo done
