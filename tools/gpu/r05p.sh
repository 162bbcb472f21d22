#!/bin/bash
# Round 5: front-loaded fragment reads in the lock-step persistent GEMM k-loop (variant builds
# libcomet_hip_front1.so: k-step 0; front2: both k-steps, DMA after the reads) and the static
# younger-half priority (COMET_GEMM_PRIO=1) against the default library: gemm / row-LN A/B/A/B,
# bench step.
#   bash tools/gpu/r05p.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
D=comet-pose-estimation_amd
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
env COMET_HIP_LIB=$D/libcomet_hip_front2.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "gemm or linear or rowln or mlp" > $O/tests_front2.log 2>&1
rc=$?; tail -2 $O/tests_front2.log; [ $rc -le 1 ] || exit 1
for r in 1 2; do
  for lib in libcomet_hip.so libcomet_hip_front1.so libcomet_hip_front2.so; do
    step env COMET_HIP_LIB=$D/$lib timeout -k 10 200 python -u tools/gemm_lib_ab.py $lib > $O/ab_$lib.$r.txt 2>&1
    step env COMET_HIP_LIB=$D/$lib timeout -k 10 200 python -u tools/rowln_lib_ab.py $lib > $O/rowln_$lib.$r.txt 2>&1
  done
  step env COMET_GEMM_PRIO=1 timeout -k 10 200 python -u tools/gemm_lib_ab.py prio > $O/ab_prio.$r.txt 2>&1
done
paste -d'\n' $O/ab_libcomet_hip.so.1.txt $O/ab_libcomet_hip_front1.so.1.txt $O/ab_libcomet_hip_front2.so.1.txt $O/ab_prio.1.txt | grep -v amdgpu.ids | cut -c1-120
paste -d'\n' $O/rowln_libcomet_hip.so.1.txt $O/rowln_libcomet_hip_front2.so.1.txt | grep -v amdgpu.ids | cut -c1-120
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  for lib in libcomet_hip.so libcomet_hip_front2.so libcomet_hip_front1.so; do
    step env COMET_HIP_LIB=$D/$lib timeout -k 10 300 $B > $O/bench_$lib.$r.json 2> $O/bench_$lib.$r.err
    python -c "import json; d=json.loads(open('$O/bench_$lib.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$lib $r', d['value'], d['ms_per_step'], k['comet_gemm']['ms_per_step'], k['comet_gemm_rowln']['ms_per_step'])"
  done
done
echo done
