# GEMM microbench vs hipBLASLt, and counter passes over one dominant shape
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gemm
mkdir -p $O
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_bench.txt 2>&1
S="74368 3072 768 1 bf16 0 20"
timeout -k 10 120 python tools/gemm_one.py $S > $O/one.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex gemm -f csv -d $O/p1 -o run -- python tools/gemm_one.py $S > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM --kernel-include-regex gemm -f csv -d $O/p2 -o run -- python tools/gemm_one.py $S > $O/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm -f csv -d $O/p3 -o run -- python tools/gemm_one.py $S > $O/p3.log 2>&1
echo done
