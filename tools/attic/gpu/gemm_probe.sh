#!/bin/bash
# GEMM probe: op tests, comet_gemm (w2 / w4 / 256-row) vs torch.matmul (hipBLASLt) per step shape, K scan
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${1:-gemm_probe}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "gemm or linear" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_bench.txt 2>&1 || exit 1
cat $O/gemm_bench.txt
bash tools/gpu/kscan.sh
