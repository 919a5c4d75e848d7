#!/bin/bash
# Fused residual + RMSNorm GEMV prologue: bit-identity tests, then single-stream decode.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or packed or hip" > gpurun_out/smallm_tests.log 2>&1 || { tail -40 gpurun_out/smallm_tests.log; exit 1; }
tail -1 gpurun_out/smallm_tests.log
timeout -k 10 500 python -u scripts/bench_latency.py --models mistral-7b llama-2-13b --prompt 512 2500 --new 256 > gpurun_out/latency_smallm.log 2>&1 || { tail -20 gpurun_out/latency_smallm.log; exit 1; }
grep -E '^\{' gpurun_out/latency_smallm.log | cut -c1-200
