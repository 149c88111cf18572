# validation + headline bench + profile
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_latent_gpu.py tests/test_row_cell_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "small_gemm or colsum or fold or latent or hyper or row" > gpurun_out/t_sel.log 2>&1; rc=$?; tail -4 gpurun_out/t_sel.log; [ $rc -eq 0 ] || exit 1
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/b_$tag.log 2>&1 || exit $?; printf "%-10s %s\n" $tag "$(tail -1 gpurun_out/b_$tag.log | cut -c150-200)"; }
run def_e X=1
run def_f X=1
for c in vae_layernorm vae_small; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --config $c > gpurun_out/b_$c.log 2>&1 || exit $?; printf "%-14s %s\n" $c "$(tail -1 gpurun_out/b_$c.log | cut -c150-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-eval > gpurun_out/prof4.log 2>&1 || exit $?
echo done
