#!/bin/bash
# Measurement pass on the GPU box: bench line (with the CPU baseline), BASELINE configs 1 and 4,
# kernel-trace stats of the bench command, per-shape GEMM census, and the kernel trace of the
# headline parity test (shows which kernel instances the parity test exercises).
#   bash tools/gpu/measure.sh <tag>        e.g. r02_v1   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
run() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
run timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
tail -c 300 $O/bench.json
run timeout -k 10 300 python bench.py --no-cpu-baseline --fwd-only > $O/fwd.json 2> $O/fwd.err
run timeout -k 10 400 python bench.py --no-cpu-baseline --batch 4 --frames 64 --image 768 --steps 2 --warmup 1 > $O/stress.json 2> $O/stress.err
run timeout -k 10 300 python tools/gemm_shapes.py > $O/gemm_shapes.txt 2> $O/gemm_shapes.err
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err
run timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_headline -o run -- python -m pytest -q -m gpu tests/test_headline_gpu.py > $O/headline_prof.log 2>&1
echo done
