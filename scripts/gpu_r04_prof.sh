#!/bin/bash
# Round-4 headline profile: rocprofv3 kernel-trace + stats of one 128-thread batch of bench.py
# (hand-written prefill GEMM default, packed-only weights, RoPE/KV write fused into decode attention).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r04
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04 -o run -- \
  python bench.py --steps 1 --warmup 0 > gpurun_out/prof_r04_bench.log 2>&1; rc=$?
tail -2 gpurun_out/prof_r04_bench.log; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py gpurun_out/prof_r04 gpurun_out/prof_r04_summary.txt > /dev/null
find gpurun_out/prof_r04 -name '*kernel_trace.csv' -delete
head -40 gpurun_out/prof_r04_summary.txt
