cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/g1; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu_tests.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu/ab2.sh step1 COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_r03a.so COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_r03a.so
