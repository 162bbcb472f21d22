#!/bin/bash
# attention: op tests, microbench (default vs opt-in v2), SQ counter passes (wave-cycle breakdown, LDS conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${1:-attn_probe}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "attn or attention" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/attn_bench.py > $O/attn_bench.txt 2>&1 || exit 1
COMET_ATTN_V2=1 timeout -k 10 120 python tools/attn_bench.py > $O/attn_bench_v2.txt 2>&1 || exit 1
cat $O/attn_bench.txt $O/attn_bench_v2.txt | grep -v amdgpu.ids
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -f csv -d $O/pmc1 -o run -- python tools/attn_bench.py > $O/pmc1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --kernel-trace -f csv -d $O/pmc2 -o run -- python tools/attn_bench.py > $O/pmc2.log 2>&1 || exit 1
python tools/sq_breakdown.py $O/pmc1 $O/pmc2
