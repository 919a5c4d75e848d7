#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "pgemm" > gpurun_out/swiglu3_tests.log 2>&1 || { tail -30 gpurun_out/swiglu3_tests.log; exit 1; }
tail -1 gpurun_out/swiglu3_tests.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --latency-rate 0 > gpurun_out/bench_swiglu.log 2>&1 || { tail -30 gpurun_out/bench_swiglu.log; exit 1; }
grep -E '^\[bench\] step|"metric"' gpurun_out/bench_swiglu.log | cut -c1-300
