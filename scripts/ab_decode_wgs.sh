#!/bin/bash
# A/B of the decode attention's split-KV target (CFC_DECODE_WGS: P = ceil(target / (B x Hkv)) balanced
# partitions per sequence) with longest-first slots, interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
for wgs in 512 2048 512 2048; do
  CFC_DECODE_WGS=$wgs timeout -k 10 400 python bench.py --steps 2 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 > gpurun_out/ab_wgs_$wgs.out 2> gpurun_out/ab_wgs_$wgs.err || exit $?
  echo "wgs=$wgs $(grep -o 'prefill=[0-9.]*s decode=[0-9.]*s' gpurun_out/ab_wgs_$wgs.err | tr '\n' ' ') $(grep -o '"value": [0-9.]*' gpurun_out/ab_wgs_$wgs.out)" | tee -a gpurun_out/r05_ab_decode_wgs.log
done
