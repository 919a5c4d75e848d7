#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd scripts && timeout -k 10 400 python -u bench_prefill_small_m.py > ../gpurun_out/smallm.log 2>&1 || { tail -20 ../gpurun_out/smallm.log; exit 1; }
grep '^{' ../gpurun_out/smallm.log
