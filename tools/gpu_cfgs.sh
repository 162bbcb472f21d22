# BASELINE configs: [2] train (default), [1] fwd-only, [4] long-sequence stress T=64 B=4 768^2
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/train.json 2> $O/train.err
timeout -k 10 400 python bench.py --no-cpu-baseline --fwd-only > $O/fwd.json 2> $O/fwd.err
timeout -k 10 600 python bench.py --no-cpu-baseline --batch 4 --frames 64 --image 768 --steps 2 --warmup 1 > $O/stress.json 2> $O/stress.err
echo done
