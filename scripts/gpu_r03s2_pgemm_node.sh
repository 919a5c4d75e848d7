#!/bin/bash
# Round 3 session 2: prefill GEMM ring variants (numerics + timing vs the library), the decoder
# prefill on pgemm, the headline with CFC_PREFILL_GEMM=hip, the node pipeline with bulk admission.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -k "pgemm or prefill_gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest_pgemm.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pgemm.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/pgemm.jsonl
timeout -k 10 300 python -u scripts/bench_pgemm.py --shapes gate_up qkv o down minilm_qkv minilm_up minilm_down bge_qkv bge_down > gpurun_out/bench_pgemm.log 2>&1; rc=$?; tail -12 gpurun_out/bench_pgemm.log; [ $rc -eq 0 ] || exit $rc
CFC_PREFILL_GEMM=hip timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench_hip_prefill.log 2>&1; rc=$?; tail -3 gpurun_out/bench_hip_prefill.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --pipeline node --steps 3 --warmup 1 > gpurun_out/bench_node.log 2>&1; rc=$?; tail -4 gpurun_out/bench_node.log; exit $rc
