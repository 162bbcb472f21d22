set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r1n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "sq_norm or cast_multi" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_model.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err
echo done
