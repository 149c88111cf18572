# split-K balance A/B for the HyperLSTM grouped launches (env overrides of ops/hyper.py)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -12 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_$tag.log 2>&1 || exit $?; printf "%-10s %s\n" $tag "$(tail -1 gpurun_out/b_$tag.log | cut -c150-200)"; }
for r in a b; do
run def_$r X=1
run sy6_$r SKR_HYP_SY=6
run sy12_$r SKR_HYP_SY=12
run sh64_$r SKR_HYP_SH=64
run both_$r SKR_HYP_SY=12 SKR_HYP_SH=64
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-eval > gpurun_out/prof3.log 2>&1 || exit $?
echo done
