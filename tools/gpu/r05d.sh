#!/bin/bash
# Round 5, fourth call: attention forward (MFMA row sums, max3 tree, permlane reductions) and
# backward (-Δ accumulator start, peeled ragged dQ tile) against the committed kernels
# (libcomet_hip_attnA.so): tests, tools/attn_bench.py A/B/A/B, bench step A/B/A, counter passes;
# the split-K row-LN path for few rows against COMET_ROWLN_NOSPLIT=1; f32 split-K (COMET_GEMM_NO_F32SPLIT=1).
#   bash tools/gpu/r05d.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn or colsum or mlp or rowln or gemm or add_rows or tokens" > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 1 2; do
  for lib in libcomet_hip.so libcomet_hip_attnA.so; do
    step env COMET_HIP_LIB=comet-pose-estimation_amd/$lib timeout -k 10 120 python -u tools/attn_bench.py > $O/attn_$lib.$r.txt 2>&1
  done
done
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
step timeout -k 10 300 $B > $O/bench_new.json 2> $O/bench_new.err
step env COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_attnA.so timeout -k 10 300 $B > $O/bench_attnA.json 2> $O/bench_attnA.err
step timeout -k 10 300 $B > $O/bench_new2.json 2> $O/bench_new2.err
step env COMET_ROWLN_NOSPLIT=1 timeout -k 10 300 $B > $O/bench_nosplit.json 2> $O/bench_nosplit.err
step env COMET_GEMM_NO_F32SPLIT=1 timeout -k 10 300 $B > $O/bench_nof32split.json 2> $O/bench_nof32split.err
step timeout -k 10 100 python -u tools/rowln_lib_ab.py split > $O/rowln_split_ab.txt 2>&1
step env COMET_ROWLN_NOSPLIT=1 timeout -k 10 100 python -u tools/rowln_lib_ab.py nosplit >> $O/rowln_split_ab.txt 2>&1
for f in bench_new bench_attnA bench_new2 bench_nosplit bench_nof32split; do
  python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"
done
step bash tools/gpu/prog_pmc.sh $TAG/pmc tools/attn_bench.py
echo done
