#!/bin/bash
# Row-LN GEMM: op parity, model-level parity through the tracker, microbenchmark, bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${1:-rowln}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k rowln > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -2 $O/ops.log
timeout -k 10 200 python -u tools/rowln_bench.py > $O/rowln_bench.txt 2>&1 || { cat $O/rowln_bench.txt; exit 1; }
COMET_ROWLN_HALF=1 timeout -k 10 200 python -u tools/rowln_bench.py > $O/rowln_bench_half.txt 2>&1 || exit 1
cat $O/rowln_bench.txt $O/rowln_bench_half.txt
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_headline_gpu.py tests/test_configs_gpu.py > $O/model.log 2>&1 || { tail -40 $O/model.log; exit 1; }
tail -2 $O/model.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
