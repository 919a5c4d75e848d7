#!/bin/bash
# Fused encoder GEMM + bias + residual + LayerNorm: numerics, then encoder batch time fused vs unfused (A/B/A/B).
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "pgemm_ln or encoder or embed" --timeout 120 --timeout-method thread > gpurun_out/pytest_pgemm_ln.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pgemm_ln.log; [ $rc -eq 0 ] || exit $rc
for f in 0 1 0 1; do
  CFC_ENCODER_LN_FUSED=$f timeout -k 10 300 python -u scripts/bench_embed.py minilm-l6 bge-small > gpurun_out/bench_embed_ln$f.log 2>&1; rc=$?; echo "fused=$f"; grep '^{' gpurun_out/bench_embed_ln$f.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
done
