set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.txt 2>&1
timeout -k 10 300 python tools/gemm_shapes.py > gpurun_out/gemm_shapes.txt 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof1 -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
