#!/bin/bash
# Headline step vs the packed prefill chunk size (tokens per prefill forward).
set -o pipefail
mkdir -p gpurun_out
for p in 32768 16384; do
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --prefill-tokens $p > gpurun_out/bench_prefill$p.log 2>&1 || { tail -5 gpurun_out/bench_prefill$p.log; exit 1; }
  echo "prefill_tokens=$p"; grep -o 'prefill=[0-9.]*s' gpurun_out/bench_prefill$p.log | tr '\n' ' '; echo; tail -1 gpurun_out/bench_prefill$p.log | cut -c1-200
done
