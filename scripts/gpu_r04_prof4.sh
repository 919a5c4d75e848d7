#!/bin/bash
# Round-4 session-3 headline profile: one 128-thread batch, no latency probe, current defaults.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "rope" > gpurun_out/rope2_tests.log 2>&1 || { tail -30 gpurun_out/rope2_tests.log; exit 1; }
tail -1 gpurun_out/rope2_tests.log
rm -rf gpurun_out/prof_r04d
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04d -o run -- \
  python bench.py --steps 1 --warmup 0 --latency-rate 0 > gpurun_out/prof_r04d_bench.log 2>&1; rc=$?
tail -2 gpurun_out/prof_r04d_bench.log; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py gpurun_out/prof_r04d gpurun_out/prof_r04d_summary.txt > /dev/null
find gpurun_out/prof_r04d -name '*kernel_trace.csv' -delete
head -36 gpurun_out/prof_r04d_summary.txt | cut -c1-200
