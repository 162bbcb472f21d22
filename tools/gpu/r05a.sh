#!/bin/bash
# Round 5, first call: settle the round-4 open measurements in one box.
#  1. the persistent GEMM's A-piece addressing: libcomet_hip.so (round-5 form: ISA identical to
#     7a6f28f^ for every instance but the 32-row one) vs libcomet_hip_wrapall.so (round-4 form),
#     row-LN and persistent-GEMM shapes, A/B/A/B;
#  2. the opt-in features' tests, then bench lines default / COMET_MLP_FUSE=1 / COMET_ROWLN_32=1 /
#     the round-4 library, default again.
#   bash tools/gpu/r05a.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
for r in 1 2; do
  for lib in libcomet_hip.so libcomet_hip_wrapall.so; do
    step env COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 120 python -u tools/rowln_lib_ab.py $lib >> $O/rowln_lib_ab.txt 2>&1
    step env COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 120 python -u tools/gemm_lib_ab.py $lib >> $O/gemm_lib_ab.txt 2>&1
  done
done
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "dact or mlp_fused or rowln" > $O/tests_optin.log 2>&1
tail -2 $O/tests_optin.log
step timeout -k 10 100 python -u tools/rowln_lib_ab.py default > $O/rowln32_ab.txt 2>&1
step env COMET_ROWLN_32=1 timeout -k 10 100 python -u tools/rowln_lib_ab.py rowln32 >> $O/rowln32_ab.txt 2>&1
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
step timeout -k 10 300 $B > $O/bench_default.json 2> $O/bench_default.err
step env COMET_MLP_FUSE=1 timeout -k 10 300 $B > $O/bench_mlpfuse.json 2> $O/bench_mlpfuse.err
step env COMET_ROWLN_32=1 timeout -k 10 300 $B > $O/bench_rowln32.json 2> $O/bench_rowln32.err
step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_wrapall.so timeout -k 10 300 $B > $O/bench_wrapall.json 2> $O/bench_wrapall.err
step timeout -k 10 300 $B > $O/bench_default2.json 2> $O/bench_default2.err
for f in bench_default bench_mlpfuse bench_rowln32 bench_wrapall bench_default2; do
  python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"
done
echo done
