#!/bin/bash
# Throughput / saturated-p50 operating curve on one GPU: threads per GPU 64 / 128 / 192 / 256,
# 3 timed steps + 1 warm-up each, throughput half only -> gpurun_out/operating_curve.log
set -o pipefail
mkdir -p gpurun_out
LOG=gpurun_out/operating_curve.log
: > $LOG
for n in 64 128 192 256; do
  cmd="python -u bench.py --threads-per-gpu $n --steps 3 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 --search-queries 0"
  echo "# $cmd" >> $LOG
  timeout -k 10 420 $cmd > gpurun_out/oc.out 2> gpurun_out/oc.err || { tail -5 gpurun_out/oc.err; exit 1; }
  tail -1 gpurun_out/oc.out >> $LOG
  grep "\[bench\]" gpurun_out/oc.err >> $LOG
  python - <<'PY'
import json
d = json.loads(open("gpurun_out/oc.out").read().strip().splitlines()[-1])
print(d["config"]["global_batch"], "threads/s", d["value"], "p50", d["p50_summary_latency_s"], flush=True)
PY
done
