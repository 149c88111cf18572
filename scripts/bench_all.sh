#!/bin/bash
# Secondary benchmarks of the framework on one MI355X (the headline is
# bench.py's default). Each line of output/*.json is one bench.py /
# bench_reference.py / bench_sample.py / bench_decode.py JSON record.
# usage (GPU box): bash scripts/bench_all.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/bench_all}
mkdir -p $out
run() { name=$1; shift; timeout -k 10 300 "$@" > $out/$name.json 2> $out/$name.err || { echo "FAILED $name"; exit 1; }; echo "$name: $(tail -1 $out/$name.json | cut -c1-160)"; }
run vae_large        python bench.py --steps 20 --warmup 3
run vae_large_fp32   python bench.py --steps 10 --warmup 2 --dtype fp32
run vae_small        python bench.py --steps 20 --warmup 3 --config vae_small
run vae_layernorm    python bench.py --steps 20 --warmup 3 --config vae_layernorm
run vae_classcond    python bench.py --steps 20 --warmup 3 --config vae_classcond
run ref_bf16         python scripts/bench_reference.py --dtype bf16
run ref_fp32         python scripts/bench_reference.py --dtype fp32
run ref_miopen_fp32  python scripts/bench_reference.py --cudnn --dtype fp32
run ref_miopen_bf16  python scripts/bench_reference.py --cudnn --dtype bf16
run sample_b128      python scripts/bench_sample.py --batch 128 --host-steps 20
run sample_b256      python scripts/bench_sample.py --batch 256 --host-steps 20
run sample_b1024     python scripts/bench_sample.py --batch 1024 --host-steps 20
run decode_ref       python scripts/bench_decode.py
