#!/bin/bash
# One capture stream per engine (warm-up and capture share the split-K workspaces): GPU tests of the
# engines / services, then the 1-step bench with both latency points.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "continuous or engine or summar or service or tp or custom_ar" > gpurun_out/capstream_tests.log 2>&1 || { tail -40 gpurun_out/capstream_tests.log; exit 1; }
tail -1 gpurun_out/capstream_tests.log
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/bench_capstream.log 2>&1 || { tail -30 gpurun_out/bench_capstream.log; exit 1; }
grep -E '"metric"' gpurun_out/bench_capstream.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['latency_mode']['p50_s'], d['latency_mode_light']['p50_s'])"
