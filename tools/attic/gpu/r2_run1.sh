#!/bin/bash
# round 2: full GPU suite + bench + kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python -u -m pytest --maxfail=10 -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/ > gpurun_out/r2_tests.log 2>&1
rc=$?
tail -40 gpurun_out/r2_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench.log 2>&1
rc=$?
tail -3 gpurun_out/r2_bench.log
exit $rc
