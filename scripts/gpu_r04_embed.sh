#!/bin/bash
# BASELINE config 2 (copilot_embedding MiniLM-L6 / BGE-small, bf16, batch 256) re-measured at HEAD.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_embed.py > gpurun_out/bench_embed_r04.log 2>&1 || { tail -25 gpurun_out/bench_embed_r04.log; exit 1; }
tail -25 gpurun_out/bench_embed_r04.log | cut -c1-300
