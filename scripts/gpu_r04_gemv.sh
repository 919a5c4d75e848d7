#!/bin/bash
# Packed GEMV rewrite (gemv_tile_kernel): numerics, the GEMV microbench, single-stream decode.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemv or rope or residual" > gpurun_out/gemv_r04g.log 2>&1 || { tail -30 gpurun_out/gemv_r04g.log; exit 1; }
tail -2 gpurun_out/gemv_r04g.log
timeout -k 10 300 python -u scripts/bench_gemv.py > gpurun_out/bench_gemv_r04g.log 2>&1 || { tail -20 gpurun_out/bench_gemv_r04g.log; exit 1; }
cut -c1-700 gpurun_out/bench_gemv_r04g.log
timeout -k 10 600 python -u scripts/bench_latency.py --models mistral-7b llama-2-13b --prompt 512 2500 --new 256 > gpurun_out/latency_r04g.log 2>&1 || { tail -20 gpurun_out/latency_r04g.log; exit 1; }
grep -E '^\{' gpurun_out/latency_r04g.log | cut -c1-200
