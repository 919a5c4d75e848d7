#!/bin/bash
# persistent prefill GEMM (variant ppp): bit-identity tests, then pps vs ppp on the four headline shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "persistent or packed_weight or packed_exact" > gpurun_out/ppp_tests.log 2>&1 || { tail -30 gpurun_out/ppp_tests.log; exit 1; }
tail -3 gpurun_out/ppp_tests.log
timeout -k 10 400 python3 -u scripts/bench_pgemm.py --shapes qkv o gate_up down --variants packed_pps packed_ppp \
  --rounds 3 --out gpurun_out/ppp_bench.jsonl > gpurun_out/ppp_bench.log 2>&1 || { tail -30 gpurun_out/ppp_bench.log; exit 1; }
cat gpurun_out/ppp_bench.jsonl
