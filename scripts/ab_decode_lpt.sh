#!/bin/bash
# A/B of longest-first decode slots (CFC_DECODE_LPT) on the full pipeline, interleaved on one box.
set -o pipefail
mkdir -p gpurun_out
for lpt in 0 1 0 1; do
  CFC_DECODE_LPT=$lpt timeout -k 10 400 python bench.py --steps 2 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 > gpurun_out/ab_lpt_$lpt.out 2> gpurun_out/ab_lpt_$lpt.err || exit $?
  echo "lpt=$lpt $(grep -o 'prefill=[0-9.]*s decode=[0-9.]*s' gpurun_out/ab_lpt_$lpt.err | tr '\n' ' ') $(grep -o '"value": [0-9.]*' gpurun_out/ab_lpt_$lpt.out)" | tee -a gpurun_out/r05_ab_decode_lpt.log
done
