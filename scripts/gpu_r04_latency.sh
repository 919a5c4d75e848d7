#!/bin/bash
# Single-stream decode (B = 1) with the round-4 packed-only weights (the GEMV reads the packed copy).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/bench_latency.py --models mistral-7b llama-2-13b --prompt 512 2500 --new 256 > gpurun_out/latency_r04.log 2>&1 || { tail -20 gpurun_out/latency_r04.log; exit 1; }
grep -E '^\{' gpurun_out/latency_r04.log | cut -c1-260
