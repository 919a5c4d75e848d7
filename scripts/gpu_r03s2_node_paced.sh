#!/bin/bash
# Node pipeline, 6 timed steps: paced source (2 steps in flight, the default) vs the whole backlog at once.
export TMPDIR=/tmp; mkdir -p gpurun_out
for n in 2 0; do
  CFC_NODE_MAX_INFLIGHT=$n timeout -k 10 400 python -u bench.py --pipeline node --steps 6 --warmup 1 > gpurun_out/bench_node_inflight$n.log 2>&1; rc=$?
  echo "max_inflight=$n"; grep "continuous engine" gpurun_out/bench_node_inflight$n.log; tail -1 gpurun_out/bench_node_inflight$n.log | cut -c1-160; grep -o '"p50_summary_latency_s": [0-9.]*' gpurun_out/bench_node_inflight$n.log; [ $rc -eq 0 ] || exit $rc
done
