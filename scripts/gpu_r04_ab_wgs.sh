#!/bin/bash
# Headline A/B on one box: decode attention partitions per (sequence, kv head) at B = 128
# (CFC_DECODE_WGS 512 -> P = 1 [default], 2048 -> P = 2, 3072 -> P = 3).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 512 2048 3072; do
  CFC_DECODE_WGS=$v timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > gpurun_out/ab_wgs_$v.log 2>&1 || { tail -30 gpurun_out/ab_wgs_$v.log; exit 1; }
  echo "== wgs=$v"; grep -E '^\[bench\] step' gpurun_out/ab_wgs_$v.log | sed 's/.*prefill=/prefill=/' | cut -c1-120
done
