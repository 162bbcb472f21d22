#!/bin/bash
# Round 5: the 32x32x16 attention forward (COMET_ATTN_FWD32=1) for D = 64 / 96 against the
# default 16x16x32 kernel after this round's forward changes: attn_bench A/B/A/B, bench step.
#   bash tools/gpu/r05s.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
TAG=${1:?tag}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $*" >&2; "$@" || { echo "step failed ($?): $*"; exit 1; }; }
for r in 1 2; do
  step timeout -k 10 120 python -u tools/attn_bench.py > $O/attn_default.$r.txt 2>&1
  step env COMET_ATTN_FWD32=1 timeout -k 10 120 python -u tools/attn_bench.py > $O/attn_fwd32.$r.txt 2>&1
done
paste -d'\n' $O/attn_default.1.txt $O/attn_fwd32.1.txt | grep -v amdgpu.ids | head -40
B="python -u bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
  step timeout -k 10 300 $B > $O/bench_default.$r.json 2> $O/bench_default.$r.err
  step env COMET_ATTN_FWD32=1 timeout -k 10 300 $B > $O/bench_fwd32.$r.json 2> $O/bench_fwd32.$r.err
  for arm in default fwd32; do
    python -c "import json; d=json.loads(open('$O/bench_$arm.$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$arm $r', d['value'], d['ms_per_step'], k['comet_attention_fwd']['ms_per_step'])"
  done
done
echo done
