# round-1 v6 measurement: full GPU tests, bench line (with CPU baseline), BASELINE configs 1 and 4,
# kernel-trace stats of the bench command and three separate PMC passes
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/v6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python bench.py --no-cpu-baseline --fwd-only > $O/fwd.json 2> $O/fwd.err
timeout -k 10 600 python bench.py --no-cpu-baseline --batch 4 --frames 64 --image 768 --steps 2 --warmup 1 > $O/stress.json 2> $O/stress.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_mfma -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc_mfma.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_fetch -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex comet -f csv -d $O/pmc_write -o run -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc_write.log 2>&1
echo done
