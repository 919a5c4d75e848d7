#!/bin/bash
# A/B of the decode GEMM's split-K slab store policy (CFC_DGEMM_SLAB_WT) in the decode step,
# interleaved runs on one box; then the numerics test of the write-through epilogue.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 -k "write_through" > gpurun_out/r05_slab_wt_test.log 2>&1 || { tail -20 gpurun_out/r05_slab_wt_test.log; exit 1; }
tail -2 gpurun_out/r05_slab_wt_test.log
for wt in 0 1 0 1 0 1; do
  CFC_DGEMM_SLAB_WT=$wt timeout -k 10 300 python bench.py --llm-only --steps 2 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 > gpurun_out/ab_wt_$wt.out 2> gpurun_out/ab_wt_$wt.err || exit $?
  echo "slab_wt=$wt $(grep -o 'prefill=[0-9.]*s decode=[0-9.]*s' gpurun_out/ab_wt_$wt.err | tr '\n' ' ')" | tee -a gpurun_out/r05_ab_slab_wt.log
done
