#!/bin/bash
# GEMM time vs K on the step's shapes (per-tile fixed cost = intercept); bias / no-bias
set -o pipefail
for K in 384 768 1536 3072; do timeout -k 5 60 python tools/gemm_one.py 74368 2304 $K 0 bf16 0 20 || exit 1; done
for K in 384 768 1536; do timeout -k 5 60 python tools/gemm_one.py 74368 2304 $K 0 bf16 0 20 nobias || exit 1; done
for K in 768 1536; do timeout -k 5 60 python tools/gemm_one.py 74368 2304 $K 1 bf16 0 20 || exit 1; done
for K in 384 768 1536 3072; do timeout -k 5 60 python tools/gemm_one.py 73728 384 $K 0 f32 1 20 || exit 1; done
for K in 384 768; do timeout -k 5 60 python tools/gemm_one.py 73728 384 $K 0 f32 1 20 nobias || exit 1; done
if [ "$1" = "test" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "gemm or linear" 2>&1 | tail -3
fi
