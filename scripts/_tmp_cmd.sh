timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; cat gpurun_out/bench_gemm.log | grep -v amdgpu.ids && \
bash scripts/gpu_check.sh pytest bench
