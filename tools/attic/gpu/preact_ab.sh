#!/bin/bash
# PREACT A/B: op parity on both libraries, GEMM microbenchmarks, bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/preact
mkdir -p $O
AB=comet-pose-estimation_amd/build_ab/libcomet_hip_ab.so
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "preact or persistent" > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -1 $O/ops.log
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_new.txt 2>&1 || exit 1
COMET_HIP_LIB=$AB timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_old.txt 2>&1 || exit 1
paste -d'\n' $O/gemm_new.txt $O/gemm_old.txt | grep -E "^ +[0-9]+ +[0-9]+ +[0-9]+ +1 " | cut -c1-70
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_new.json 2>/dev/null || exit 1
COMET_HIP_LIB=$AB timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_old.json 2>/dev/null || exit 1
for f in b_new b_old; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'])"; done
