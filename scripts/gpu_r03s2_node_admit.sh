#!/bin/bash
# Node pipeline admission A/B: full-batch first admission (default) vs earlier, smaller admissions.
export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "128 3000" "64 500" "32 200"; do
  set -- $cfg
  CFC_NODE_MIN_ADMIT=$1 CFC_NODE_ADMIT_WAIT_MS=$2 timeout -k 10 300 python -u bench.py --pipeline node --steps 3 --warmup 1 > gpurun_out/bench_node_admit_$1.log 2>&1; rc=$?
  echo "min_admit=$1 wait=$2"; grep "continuous engine" gpurun_out/bench_node_admit_$1.log; tail -1 gpurun_out/bench_node_admit_$1.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
