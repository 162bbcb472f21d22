#!/bin/bash
# round 2: re-run the previously failing GPU tests, then the bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_configs_gpu.py tests/test_headline_gpu.py \
  "tests/test_model_gpu.py::test_e2e_bf16_grads_match_reference_bf16" \
  "tests/test_model_gpu.py::test_dead_row_pruning_is_output_identical" \
  "tests/test_ops_gpu.py::test_cast_multi_and_weight_cache_refresh" > gpurun_out/r2_tests2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|max diff|max err|spread|^E " gpurun_out/r2_tests2.log | head -60
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench.log 2>&1 || exit $?
tail -2 gpurun_out/r2_bench.log
exit $rc
