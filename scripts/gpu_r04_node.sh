#!/bin/bash
# Round-4: the node pipeline (the deployment's services, continuous engine) vs the bench pipeline on
# one box, 4 timed steps each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 --latency-rate 0 > gpurun_out/r04_bench4.log 2>&1 || { tail -20 gpurun_out/r04_bench4.log; exit 1; }
grep -E '^\[bench\] step|"metric"' gpurun_out/r04_bench4.log | cut -c1-330
timeout -k 10 600 python -u bench.py --pipeline node --steps 4 --warmup 1 > gpurun_out/r04_node4.log 2>&1 || { tail -20 gpurun_out/r04_node4.log; exit 1; }
grep -E 'step|"metric"|engine' gpurun_out/r04_node4.log | cut -c1-330
