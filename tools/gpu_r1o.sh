set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r1o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_model.log 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
