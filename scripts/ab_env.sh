#!/bin/bash
# Interleaved A/B of the headline bench over values of one environment switch, on one box.
#   scripts/ab_env.sh VAR "A B" [ROUNDS=2] [-- extra bench.py args]
# e.g. ab_env.sh CFC_DECODE_LPT "0 1"; ab_env.sh CFC_DECODE_WGS "512 2048"; ab_env.sh CFC_PREP_MARGIN
# "2.0 1.25" 2 -- --steps 20 --warmup 5 (the round-5 ab_decode_lpt / ab_decode_wgs / ab_prep_margin /
# ab_qkv_split / ab_slab_wt runs).  Default bench args: 2 timed steps + 1 warm-up, throughput half
# only.  One line per run: value, prefill / decode seconds per batch, p50 -> gpurun_out/ab_<VAR>.log
set -o pipefail
VAR=$1; VALUES=$2; ROUNDS=${3:-2}
shift 3 2>/dev/null || shift $#
[ "$1" = "--" ] && shift
ARGS=${*:-"--steps 2 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 --search-queries 0"}
mkdir -p gpurun_out
LOG=gpurun_out/ab_$VAR.log
for r in $(seq 1 "$ROUNDS"); do
  for v in $VALUES; do
    env "$VAR=$v" timeout -k 10 600 python -u bench.py $ARGS > gpurun_out/ab.out 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python - "$VAR=$v" >> "$LOG" <<'PY'
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
