#!/bin/bash
# round-2 parity tests on the GPU box (one pytest process, per-test timeouts)
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_headline_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py > gpurun_out/r2_tests.log 2>&1
rc=$?
tail -60 gpurun_out/r2_tests.log
exit $rc
