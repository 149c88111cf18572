set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --trace > gpurun_out/t_bf16.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --trace --no-graph > gpurun_out/t_bf16_eager.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --trace --dtype fp32 > gpurun_out/t_fp32.log 2>&1
grep cost gpurun_out/t_bf16.log | grep -v metric | tr '\n' ' '; echo
grep cost gpurun_out/t_bf16_eager.log | grep -v metric | tr '\n' ' '; echo
grep cost gpurun_out/t_fp32.log | grep -v metric | tr '\n' ' '; echo
