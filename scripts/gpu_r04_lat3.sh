#!/bin/bash
# Single-stream decode after the 8-at-a-time slab sums (reduce / RoPE from slabs); fused-RoPE A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/latprof3 -o lat -- python3 -u scripts/bench_latency.py --models mistral-7b --prompt 512 --new 128 --reps 1 > gpurun_out/latprof3.log 2>&1 || { tail -20 gpurun_out/latprof3.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/latprof3 > gpurun_out/latprof3.txt && cut -c1-200 gpurun_out/latprof3.txt
CFC_DECODE_ROPE_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/latprof4 -o lat -- python3 -u scripts/bench_latency.py --models mistral-7b --prompt 512 --new 128 --reps 1 > gpurun_out/latprof4.log 2>&1 || { tail -20 gpurun_out/latprof4.log; exit 1; }
grep -E "^\{" gpurun_out/latprof3.log gpurun_out/latprof4.log | cut -c1-200
python3 scripts/prof_summary.py gpurun_out/latprof4 > gpurun_out/latprof4.txt && cut -c1-200 gpurun_out/latprof4.txt
