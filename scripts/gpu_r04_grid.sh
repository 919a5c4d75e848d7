#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd scripts && timeout -k 10 400 python -u bench_gemv_grid.py > ../gpurun_out/gemv_grid.log 2>&1 || { tail -20 ../gpurun_out/gemv_grid.log; exit 1; }
cat ../gpurun_out/gemv_grid.log
