#!/bin/bash
# persistent GEMM: per-tile fixed cost with and without the C stores (diagnostic)
set -o pipefail
for K in 384 768 1536 3072; do timeout -k 5 60 python tools/gemm_one.py 74368 2304 $K 0 bf16 0 20 || exit 1; done
export COMET_GEMM_DIAG_NOSTORE=1
for K in 384 768 1536 3072; do timeout -k 5 60 python tools/gemm_one.py 74368 2304 $K 0 bf16 0 20 || exit 1; done
for K in 384 768 1536; do timeout -k 5 60 python tools/gemm_one.py 73728 384 $K 0 f32 1 20 || exit 1; done
