#!/bin/bash
# Kernel breakdown of single-stream Mistral-7B decode (packed-only weights).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/latprof -o lat -- python3 -u scripts/bench_latency.py --models mistral-7b --prompt 512 --new 128 --reps 1 > gpurun_out/latprof.log 2>&1 || { tail -20 gpurun_out/latprof.log; exit 1; }
grep -E '^\{' gpurun_out/latprof.log | cut -c1-200
python3 scripts/prof_summary.py gpurun_out/latprof | cut -c1-230
