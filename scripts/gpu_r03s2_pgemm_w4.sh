#!/bin/bash
# Prefill GEMM: numerics of every K-loop variant, then timing of the 4-wave 128x128 variants vs the library.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k pgemm --timeout 120 --timeout-method thread > gpurun_out/pytest_pgemm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pgemm.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/pgemm.jsonl
timeout -k 10 400 python -u scripts/bench_pgemm.py --shapes gate_up qkv o down minilm_qkv minilm_down bge_qkv bge_down > gpurun_out/bench_pgemm.log 2>&1; rc=$?; tail -12 gpurun_out/bench_pgemm.log; exit $rc
