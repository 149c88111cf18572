set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
SKR_GEMM_AREG=1 timeout -k 10 300 python -m pytest tests -m gpu -q -x -k "skinny or grouped or hyper" > gpurun_out/areg_tests.log 2>&1; rc=$?; tail -3 gpurun_out/areg_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
SKR_GEMM_AREG=1 BENCH_TAG=areg bash scripts/gpu_check.sh bench_env || exit $?
BENCH_TAG=base bash scripts/gpu_check.sh bench_env || exit $?
