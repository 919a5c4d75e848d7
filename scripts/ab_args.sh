#!/bin/bash
# Interleaved A/B of the headline bench over two bench.py argument sets, on one box.
#   scripts/ab_args.sh "ARGS_A" "ARGS_B" [ROUNDS=2]
# Both arms add: 3 timed steps + 1 warm-up, throughput half only.  One line per run: arm, value,
# prefill / decode seconds per batch, p50 -> gpurun_out/ab_args.log
set -o pipefail
A=$1; B=$2; ROUNDS=${3:-2}
BASE="--steps 3 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 --search-queries 0"
mkdir -p gpurun_out
LOG=gpurun_out/ab_args.log
for r in $(seq 1 "$ROUNDS"); do
  for arm in A B; do
    if [ $arm = A ]; then X=$A; else X=$B; fi
    timeout -k 10 600 python -u bench.py $BASE $X > gpurun_out/ab.out 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python - "$arm [$X]" >> "$LOG" <<'PY'
import json, re, sys
d = json.loads(open("gpurun_out/ab.out").read().strip().splitlines()[-1])
err = open("gpurun_out/ab.err").read()
pf = [float(x) for x in re.findall(r"\bprefill=([0-9.]+)s", err)]
dc = [float(x) for x in re.findall(r"\bdecode=([0-9.]+)s", err)]
print(f"{sys.argv[1]} value={d['value']} p50={d['p50_summary_latency_s']} prefill={pf} decode={dc}", flush=True)
PY
    tail -1 "$LOG"
  done
done
