# final validation: full GPU suite, smoke, headline bench (twice)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?; tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1 || exit $?; tail -1 gpurun_out/b_default.log | cut -c1-260
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_final.log 2>&1 || exit $?; tail -1 gpurun_out/b_final.log | cut -c150-200
echo done
