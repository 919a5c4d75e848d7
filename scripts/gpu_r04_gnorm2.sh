#!/bin/bash
# Fused-norm GEMV with the prologue's first loads ahead of the weights: tests, then single-stream
# decode at 8 and 4 waves, and the unfused path, on one box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemv or fused_norm or residual" > gpurun_out/gnorm2_tests.log 2>&1 || { tail -40 gpurun_out/gnorm2_tests.log; exit 1; }
tail -1 gpurun_out/gnorm2_tests.log
for cfg in "CFC_GEMV_NORM_WAVES=8" "CFC_GEMV_NORM_WAVES=4" "CFC_DECODE_GEMV_NORM=0"; do
  env $cfg timeout -k 10 300 python -u scripts/bench_latency.py --models mistral-7b llama-2-13b --prompt 512 --new 256 > gpurun_out/lat_$cfg.log 2>&1 || { tail -20 gpurun_out/lat_$cfg.log; exit 1; }
  echo "== $cfg"; grep -E '^\{' gpurun_out/lat_$cfg.log | cut -c1-150
done
