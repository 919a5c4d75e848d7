#!/bin/bash
# Round-4: node pipeline with the continuous summarizer's idle / deliver counters.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --pipeline node --steps 4 --warmup 1 > gpurun_out/r04_node4b.log 2>&1 || { tail -20 gpurun_out/r04_node4b.log; exit 1; }
grep -E 'step|"metric"|engine' gpurun_out/r04_node4b.log | cut -c1-400
