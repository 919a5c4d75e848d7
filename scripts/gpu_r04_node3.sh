#!/bin/bash
# Round-4: node pipeline with 3 steps in flight (upstream gets two decode batches of lead time).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFC_NODE_MAX_INFLIGHT=3 timeout -k 10 600 python -u bench.py --pipeline node --steps 4 --warmup 1 > gpurun_out/r04_node4c.log 2>&1 || { tail -20 gpurun_out/r04_node4c.log; exit 1; }
grep -E 'step|"metric"|engine' gpurun_out/r04_node4c.log | cut -c1-400
