set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "attention" > $O/pytest_attn.log 2>&1
timeout -k 10 300 python tools/attn_bench.py > $O/attn_new.txt 2>&1
COMET_ATTN_WPE=3 COMET_ATTN_BWD_G1=1 timeout -k 10 300 python tools/attn_bench.py > $O/attn_wpe3.txt 2>&1
COMET_ATTN_WPE=1 timeout -k 10 300 python tools/attn_bench.py > $O/attn_wpe1.txt 2>&1
COMET_ATTN_QG1=1 timeout -k 10 300 python tools/attn_bench.py > $O/attn_qg1.txt 2>&1
COMET_ATTN_V1=1 COMET_ATTN_BWD_V1=1 timeout -k 10 300 python tools/attn_bench.py > $O/attn_v1.txt 2>&1
