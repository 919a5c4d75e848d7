#!/bin/bash
# The headline as the driver runs it: 20 timed steps after 5 warm-up steps, latency probes after.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1 || { tail -30 gpurun_out/bench20.log; exit 1; }
grep -E '"metric"' gpurun_out/bench20.log | cut -c1-1500
