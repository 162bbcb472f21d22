set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pp
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "gemm" --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_bench.txt 2>&1
echo done
