#!/bin/bash
# A/B of the XCD-local prefill attention grid (CFC_PREFILL_XCD=0 / 1) + prefill numerics tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "prefill or attention or engine" --timeout 120 --timeout-method thread > gpurun_out/pytest_prefill.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_prefill.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1 0 1; do
  CFC_PREFILL_XCD=$x timeout -k 10 300 python scripts/bench_attn.py > gpurun_out/attn_xcd$x.log 2>&1 || exit 1
  echo "XCD=$x"; grep prefill gpurun_out/attn_xcd$x.log
done
