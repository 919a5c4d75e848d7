#!/bin/bash
# The bench's light-load latency point (0.5 threads/s, 12 threads) next to the 8/s one.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/bench_light.log 2>&1 || { tail -30 gpurun_out/bench_light.log; exit 1; }
grep -E '"metric"' gpurun_out/bench_light.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['latency_mode'], d['latency_mode_light'])"
