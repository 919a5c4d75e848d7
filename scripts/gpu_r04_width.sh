#!/bin/bash
# Continuous engine with width-bucketed decode graphs: GPU tests, then the bench (1 step) with
# both latency points.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "continuous or engine or summar or service or tp" > gpurun_out/width_tests.log 2>&1 || { tail -40 gpurun_out/width_tests.log; exit 1; }
tail -1 gpurun_out/width_tests.log
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/bench_width.log 2>&1 || { tail -30 gpurun_out/bench_width.log; exit 1; }
grep -E '"metric"' gpurun_out/bench_width.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['latency_mode'], d['latency_mode_light'])"
