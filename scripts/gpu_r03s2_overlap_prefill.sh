#!/bin/bash
# Prefill of batch i+1 on half the CUs beside batch i's decode: engine numerics, then the headline
# bench with and without it on the same box (off, on, off, on).
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_engine_overlap.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_engine_overlap.log; [ $rc -eq 0 ] || exit $rc
for mode in on off; do
  timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --overlap-prefill $mode > gpurun_out/bench_overlap_$mode.log 2>&1; rc=$?
  echo "overlap-prefill=$mode"; grep "^\[bench\] step" gpurun_out/bench_overlap_$mode.log | cut -c1-200; tail -1 gpurun_out/bench_overlap_$mode.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
