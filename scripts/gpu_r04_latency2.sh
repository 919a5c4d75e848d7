#!/bin/bash
# Packed GEMV at 8 waves x 16 fragments in flight: numerics, then single-stream decode again.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemv" > gpurun_out/gemv_r04b.log 2>&1 || { tail -30 gpurun_out/gemv_r04b.log; exit 1; }
tail -2 gpurun_out/gemv_r04b.log
timeout -k 10 600 python -u scripts/bench_latency.py --models mistral-7b llama-2-13b --prompt 512 2500 --new 256 > gpurun_out/latency_r04b.log 2>&1 || { tail -20 gpurun_out/latency_r04b.log; exit 1; }
grep -E '^\{' gpurun_out/latency_r04b.log | cut -c1-260
