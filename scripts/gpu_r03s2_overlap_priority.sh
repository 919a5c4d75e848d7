#!/bin/bash
# Prefill beside decode with stream priorities instead of CU masks (whole chip, decode first).
export TMPDIR=/tmp; mkdir -p gpurun_out
CFC_OVERLAP_MODE=priority timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --overlap-prefill on > gpurun_out/bench_overlap_priority.log 2>&1; rc=$?
grep "^\[bench\] step" gpurun_out/bench_overlap_priority.log | cut -c1-200; tail -1 gpurun_out/bench_overlap_priority.log | cut -c1-200; exit $rc
