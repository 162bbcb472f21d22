# tests + bench + kernel-trace stats of the same bench command
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof3 -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err
echo done
