set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc3
mkdir -p $O
S="74368 3072 3072 0 bf16 0 10"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
timeout -k 10 120 python tools/gemm_one.py $S > $O/one.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-include-regex "gemm" -f csv -d $O/a1 -o run -- python tools/gemm_one.py $S > $O/a1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc $P2 --kernel-include-regex "gemm" -f csv -d $O/a2 -o run -- python tools/gemm_one.py $S > $O/a2.log 2>&1
echo done
