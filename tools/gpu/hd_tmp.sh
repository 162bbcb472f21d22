cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/st13; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "rowln or persistent or gemm" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit 1
for sh in "65536 384 384 ln_norm2" "65536 384 1536 ln_dual_ctx" "74368 768 768 0 f32 1" "74368 768 3072 0 f32 1"; do
  COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_stamp.so timeout -k 10 60 python -u tools/gemm_stamps.py $sh >> $O/stamps.txt 2>&1 || { echo "stamps failed $sh"; tail $O/stamps.txt; exit 1; }
done
grep -v "amdgpu.ids" $O/stamps.txt
for l in libcomet_hip_r03b.so libcomet_hip.so libcomet_hip_r03b.so libcomet_hip.so; do COMET_HIP_LIB=comet-pose-estimation_amd/$l timeout -k 10 120 python tools/rowln_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$l /"; done
bash tools/gpu/lib_ab.sh ab5 libcomet_hip_r03b.so libcomet_hip.so | grep float32
bash tools/gpu/ab2.sh step2 COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_r03b.so COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_r03b.so
