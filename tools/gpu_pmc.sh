# Round-1 measurement run on the GPU box: tests, bench line, kernel-trace stats of the same
# bench command, and three separate PMC passes (MFMA busy, FETCH_SIZE, WRITE_SIZE) over it.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof2 -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_mfma -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc_mfma.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc_write.log 2>&1
echo done
