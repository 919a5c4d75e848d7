#!/bin/bash
# Headline evidence on one box: rocprofv3 kernel stats of one batch, then the bench as the driver
# runs it (20 timed steps + 5 warm-up, latency points, search latency).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps 1 --warmup 0 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 --search-queries 0 > gpurun_out/prof_bench.log 2>&1 || { tail -5 gpurun_out/prof_bench.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof gpurun_out/r06_prof_full_bench.txt > /dev/null
find gpurun_out/prof -name '*kernel_trace.csv' -delete
head -16 gpurun_out/r06_prof_full_bench.txt | cut -c1-150
timeout -k 10 650 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_20steps.out 2> gpurun_out/r06_bench_20steps.err || { tail -5 gpurun_out/r06_bench_20steps.err; exit 1; }
tail -1 gpurun_out/r06_bench_20steps.out
