#!/bin/bash
# Llama-3-70B bf16 on one MI355X (BASELINE config 5 without TP): throughput vs threads per GPU.
set -o pipefail
mkdir -p gpurun_out
for b in 96; do
  timeout -k 10 900 python bench.py --model llama-3-70b --threads-per-gpu $b --kv-max-prompt 3072 --steps 1 --warmup 1 > gpurun_out/bench_70b_b$b.log 2>&1 || { tail -5 gpurun_out/bench_70b_b$b.log; exit 1; }
  tail -2 gpurun_out/bench_70b_b$b.log | cut -c1-400
done
