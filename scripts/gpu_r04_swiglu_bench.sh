#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --latency-rate 0 > gpurun_out/bench_instr.log 2>&1 || { tail -30 gpurun_out/bench_instr.log; exit 1; }
grep -E '^\[bench\] step|"metric"' gpurun_out/bench_instr.log | cut -c1-300
