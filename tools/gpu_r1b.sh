# tests + bench + kernel-trace stats of the same bench command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/attn_bench.py > $O/attn_bench.txt 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_full.json 2> $O/bench_full.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof3 -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err
