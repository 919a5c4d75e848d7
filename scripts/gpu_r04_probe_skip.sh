#!/bin/bash
# PROBE: decode time with the batch's shared prefix blocks skipped by the attention (wrong tokens,
# timing only) vs read -- the most a shared-prefix (cascade) attention could save.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  CFC_PROBE_SKIP_SHARED=$v timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > gpurun_out/probe_skip_$v.log 2>&1 || { tail -30 gpurun_out/probe_skip_$v.log; exit 1; }
  echo "== skip=$v"; grep -E '^\[bench\] step' gpurun_out/probe_skip_$v.log | cut -c1-260
done
