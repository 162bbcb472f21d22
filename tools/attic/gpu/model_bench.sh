#!/bin/bash
# Model-level GPU parity tests (e2e goldens, headline, configs, ablations, data, metrics) + bench line.
#   bash tools/gpu/model_bench.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_model_gpu.py \
  tests/test_headline_gpu.py tests/test_configs_gpu.py tests/test_ablation_gpu.py > $O/model.log 2>&1 || { tail -40 $O/model.log; exit 1; }
tail -2 $O/model.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
