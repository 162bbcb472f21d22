#!/bin/bash
# Round 5: the DDP simulated-ranks test with per-key prints (and the second local pass), then
# the asm-LDS-DMA persistent GEMM (libcomet_hip_asmdma.so) against the default library:
# tools/gemm_lib_ab.py A/B/A/B and the bench step A/B/A.
#   bash tools/gpu/r05h.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread "tests/test_configs_gpu.py::test_ddp_simulated_ranks_equal_B2_gradients[headline]" > $O/ddp.log 2>&1
echo "ddp rc $?"; grep -E "rel-to-max|passed|failed" $O/ddp.log | head -40
for r in 1 2; do
  for lib in libcomet_hip.so libcomet_hip_asmdma.so; do
    step env COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 200 python -u tools/gemm_lib_ab.py $lib > $O/ab_$lib.$r.txt 2>&1
  done
done
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
step timeout -k 10 300 $B > $O/bench_a.json 2> $O/bench_a.err
step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_asmdma.so timeout -k 10 300 $B > $O/bench_b.json 2> $O/bench_b.err
step timeout -k 10 300 $B > $O/bench_a2.json 2> $O/bench_a2.err
for f in bench_a bench_b bench_a2; do
  python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['kernels']['comet_gemm']['ms_per_step'], d['kernels']['comet_gemm_rowln']['ms_per_step'])"
done
paste $O/ab_libcomet_hip.so.1.txt $O/ab_libcomet_hip_asmdma.so.1.txt | head -30
echo done
