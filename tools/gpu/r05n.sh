#!/bin/bash
# Round 5: the ping-pong k-loop of the 256 x 256 persistent GEMM (libcomet_hip_ping.so,
# COMET_GEMM_PING=1) -- GEMM op tests, gemm_lib_ab.py A/B/A/B against the default library (and the
# refactored default path of the new library), the bench step A/B/A.
#   bash tools/gpu/r05n.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
NEW=comet-pose-estimation_amd/libcomet_hip_ping.so
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step env COMET_HIP_LIB=$NEW COMET_GEMM_PING=1 timeout -k 10 200 python -u tools/gemm_lib_ab.py ping > $O/ab_ping.0.txt 2>&1
grep -v amdgpu.ids $O/ab_ping.0.txt
env COMET_HIP_LIB=$NEW COMET_GEMM_PING=1 timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "gemm or linear or mlp" > $O/tests_ping.log 2>&1
rc=$?; tail -3 $O/tests_ping.log; [ $rc -le 1 ] || exit 1
for r in 1 2; do
  step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip.so timeout -k 10 200 python -u tools/gemm_lib_ab.py old > $O/ab_old.$r.txt 2>&1
  step env COMET_HIP_LIB=$NEW timeout -k 10 200 python -u tools/gemm_lib_ab.py new_noping > $O/ab_new.$r.txt 2>&1
  step env COMET_HIP_LIB=$NEW COMET_GEMM_PING=1 timeout -k 10 200 python -u tools/gemm_lib_ab.py ping > $O/ab_ping.$r.txt 2>&1
done
paste -d'\n' $O/ab_old.1.txt $O/ab_new.1.txt $O/ab_ping.1.txt | grep -v amdgpu.ids | cut -c1-140
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip.so timeout -k 10 300 $B > $O/bench_old.json 2> $O/bench_old.err
step env COMET_HIP_LIB=$NEW COMET_GEMM_PING=1 timeout -k 10 300 $B > $O/bench_ping.json 2> $O/bench_ping.err
step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip.so timeout -k 10 300 $B > $O/bench_old2.json 2> $O/bench_old2.err
step env COMET_HIP_LIB=$NEW COMET_GEMM_PING=1 timeout -k 10 300 $B > $O/bench_ping2.json 2> $O/bench_ping2.err
for f in bench_old bench_ping bench_old2 bench_ping2; do
  python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); k=d['kernel_instances']; print('$f', d['value'], d['ms_per_step'], d['kernels']['comet_gemm']['ms_per_step'], k.get('comet_gemm|pp256x256.L00.bf16',{}).get('ms_per_step'), k.get('comet_gemm|pp256x256.L00.f32',{}).get('ms_per_step'))"
done

timeout -k 10 400 python -u -m pytest -x -q -s --timeout 380 --timeout-method thread "tests/test_configs_gpu.py::test_ddp_simulated_ranks_equal_B2_gradients[headline]" > $O/ddp.log 2>&1
echo "ddp rc $?"; grep -E "pre-reduce|passed|failed|Error" $O/ddp.log | head -30
echo done
