#!/bin/bash
# GPU validation session for gpurun: each step has its own time limit; a
# crash / abort / timeout (anything other than a clean pass or an ordinary
# test failure) ends the session so nothing else touches the GPU.
# usage: scripts/gpu_check.sh [pytest|smoke|bench|prof ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(pytest smoke bench)

run() {  # name, limit, cmd...
    local name=$1 lim=$2
    shift 2
    echo "== $name (limit ${lim}s): $*"
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== aborting session after $name (rc=$rc)"
        exit $rc
    fi
    return 0
}

for s in "${steps[@]}"; do
    case $s in
        pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread ;;
        pytest_sel) run pytest_sel 600 python -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method thread -k "${PYTEST_K:-fused}" ;;
        pytest_file) run pytest_file 600 python -u -m pytest "${PYTEST_FILE:-tests/test_persist_gpu.py}" -m gpu -v -x --timeout 240 --timeout-method thread ;;
        bench_env) run "bench_${BENCH_TAG:-env}" 600 python bench.py --steps 10 --warmup 2 ;;
        bench_vae_miopen) run bench_vae_miopen 600 python scripts/bench_vae_miopen.py --config vae_small --dtype bf16 ;;
        bench_vae_miopen_fp32) run bench_vae_miopen_fp32 600 python scripts/bench_vae_miopen.py --config vae_small --dtype fp32 ;;
        cli_vae_train) run cli_vae_train 600 python -m sketch_rnn_amd.cli.vae_train --preset vae_large --synthetic 2000 --num_steps 80 --log_every 20 --save_every 0 --save_dir /tmp/skr_cli_vae --metrics gpurun_out/cli_vae_train_metrics.jsonl ;;
        bench_dp1) run bench_dp1 600 python scripts/bench_dp1.py ;;
        bench_wgrad) run bench_wgrad 600 python scripts/bench_wgrad.py ;;
        bench_gemm) run bench_gemm 600 python scripts/bench_gemm.py ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py --steps 10 --warmup 2 ;;
        bench_fp32) run bench_fp32 600 python bench.py --steps 5 --warmup 2 --dtype fp32 ;;
        bench_classcond) run bench_classcond 600 python bench.py --steps 10 --warmup 2 --config vae_classcond ;;
        bench_layernorm) run bench_layernorm 600 python bench.py --steps 10 --warmup 2 --config vae_layernorm ;;
        bench_small) run bench_small 600 python bench.py --steps 10 --warmup 2 --config vae_small ;;
        bench_torch) run bench_torch 900 python bench.py --steps 3 --warmup 1 --backend torch --no-eval ;;
        bench_torch_small) run bench_torch_small 600 python bench.py --steps 3 --warmup 1 --backend torch --no-eval --config vae_small ;;
        bench_sample) run bench_sample 600 python scripts/bench_sample.py ;;
        bench_sample_1k) run bench_sample_1k 600 python scripts/bench_sample.py --batch 1024 ;;
        sample_f1) for bb in 128 1024; do run sample_b${bb}_bf16 300 python scripts/bench_sample.py --batch $bb --host-steps 2; done ;;
        prof_small) run prof_small 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-eval --config vae_small ;;
        prof_ln) run prof_ln 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ln -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-eval --config vae_layernorm ;;
        bench_wide_gemm) run bench_wide_gemm 300 python scripts/bench_wide_gemm.py ;;
        pmc_fetch) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-eval ;;
        pmc_write) run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-eval ;;
        converge_a) run converge_a 1100 python scripts/converge.py --config vae_large --steps 2000 --seeds 0,1 --arms hip-bf16,hip-fp32 --out gpurun_out/converge_large_r5.jsonl ;;
        converge_b) run converge_b 1100 python scripts/converge.py --config vae_large --steps 2000 --seeds 2 --arms hip-bf16,hip-fp32 --out gpurun_out/converge_large_r5_s2.jsonl ;;
        bench_b128) run bench_b128 600 python bench.py --steps 10 --warmup 2 --batch 128 ;;
        prof_sample_fused) run prof_sample_fused 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sample_fused -o run --output-format csv -- python scripts/bench_sample.py --batch 128 --reps 1 --host-steps 2 ;;
        bench_ref) run bench_ref 600 python scripts/bench_reference.py ;;
        bench_ref_bf16) run bench_ref_bf16 600 python scripts/bench_reference.py --dtype bf16 ;;
        bench_ref_torch) run bench_ref_torch 600 python scripts/bench_reference.py --backend torch --steps 5 ;;
        bench_ref_cudnn) run bench_ref_cudnn 600 python scripts/bench_reference.py --cudnn ;;
        prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-eval ;;
        dp_rehearsal) run dp_rehearsal 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo --config vae_small ;;
        dp_rehearsal_noov) SKR_DP_OVERLAP=0 run dp_rehearsal_noov 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo --config vae_small ;;
        dp_rehearsal_nograph) run dp_rehearsal_nograph 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 3 --warmup 2 --dist-backend gloo --config vae_small --no-graph ;;
        prof_ref) run prof_ref 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref -o run --output-format csv -- python scripts/bench_reference.py --dtype bf16 --steps 5 --warmup 2 ;;
        prof_sample) run prof_sample 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sample -o run --output-format csv -- python scripts/bench_sample.py --reps 1 --host-steps 2 ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "== session done"
