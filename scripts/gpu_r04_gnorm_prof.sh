#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gnprof -o lat -- python3 -u scripts/bench_latency.py --models mistral-7b --prompt 512 --new 128 --reps 1 > gpurun_out/gnprof.log 2>&1 || { tail -20 gpurun_out/gnprof.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/gnprof > gpurun_out/gnprof.txt && cut -c1-180 gpurun_out/gnprof.txt
