set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for tag in a b; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_fast_$tag.log 2>&1 || exit $?; tail -1 gpurun_out/b_fast_$tag.log | cut -c1-200
SKR_HIP_LIB=$PWD/sketch_rnn_amd/_lib/variants/libskrnn_hip_exact_act.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_exact_$tag.log 2>&1 || exit $?; tail -1 gpurun_out/b_exact_$tag.log | cut -c1-200
SKR_ROW_CELLS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_norow_$tag.log 2>&1 || exit $?; tail -1 gpurun_out/b_norow_$tag.log | cut -c1-200
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --config vae_layernorm > gpurun_out/b_ln.log 2>&1 || exit $?; tail -1 gpurun_out/b_ln.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fast -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-eval > gpurun_out/prof_fast.log 2>&1 || exit $?
echo done
