#!/bin/bash
# A/B of the prefill chunk size (rows per packed prefill call) on the full pipeline, interleaved.
set -o pipefail
mkdir -p gpurun_out
for pt in 16384 32768 16384 32768; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --prefill-tokens $pt --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 > gpurun_out/ab_pt_$pt.out 2> gpurun_out/ab_pt_$pt.err || exit $?
  echo "prefill_tokens=$pt $(grep -o 'prefill=[0-9.]*s decode=[0-9.]*s' gpurun_out/ab_pt_$pt.err | tr '\n' ' ') $(grep -o '"value": [0-9.]*' gpurun_out/ab_pt_$pt.out)" | tee -a gpurun_out/r05_ab_prefill_chunk.log
done
