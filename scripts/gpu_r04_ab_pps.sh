#!/bin/bash
# Headline A/B on one box: prefill K loop pp vs pps (2 timed steps each).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in pp pps; do
  CFC_PGEMM_VARIANT=$v timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > gpurun_out/ab_$v.log 2>&1 || { tail -30 gpurun_out/ab_$v.log; exit 1; }
  echo "== $v"; grep -E '^\[bench\] step' gpurun_out/ab_$v.log | cut -c1-260
done
