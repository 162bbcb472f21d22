#!/bin/bash
# Round 5, second call: the swizzled / LDS-DMA attention kernels (tests, A/B against the round-4
# kernels: libcomet_hip_attnr4.so), the bench line with 32-row row-LN tiles by default, the fused-MLP
# bench line, and the configs[3] per-rank (B = 8) simulated-ranks test.
#   bash tools/gpu/r05b.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn or rowln" > $O/tests_attn.log 2>&1
tail -2 $O/tests_attn.log
for r in 1 2; do
  for lib in libcomet_hip.so libcomet_hip_attnr4.so; do
    step env COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 120 python -u tools/attn_bench.py > $O/attn_$lib.$r.txt 2>&1
  done
done
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
step timeout -k 10 300 $B > $O/bench_default.json 2> $O/bench_default.err
step env COMET_MLP_FUSE=1 timeout -k 10 300 $B > $O/bench_mlpfuse.json 2> $O/bench_mlpfuse.err
step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_attnr4.so timeout -k 10 300 $B > $O/bench_attnr4.json 2> $O/bench_attnr4.err
step timeout -k 10 300 $B > $O/bench_default2.json 2> $O/bench_default2.err
for f in bench_default bench_mlpfuse bench_attnr4 bench_default2; do
  python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"
done
step timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_configs_gpu.py -k "simulated_ranks and headline_B8" -s > $O/tests_ddp_b8.log 2>&1
tail -3 $O/tests_ddp_b8.log
echo done
