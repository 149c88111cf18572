mkdir -p gpurun_out
timeout -k 10 120 ./bin/cell_bench 200 > gpurun_out/cell_bench.txt 2>&1 || exit $?
cat gpurun_out/cell_bench.txt
bash scripts/gpu_check.sh pytest bench
