set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r1j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "attention or attn" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
