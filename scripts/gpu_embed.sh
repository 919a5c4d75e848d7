#!/bin/bash
# Encoder path on one GPU: numerics tests of the encoder kernels, the BASELINE config-2 embedding
# benchmark, and a rocprofv3 kernel breakdown of it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "encoder or embed or hf or knn or layernorm" --timeout 120 --timeout-method thread > gpurun_out/pytest_embed.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_embed.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_embed.py > gpurun_out/bench_embed.log 2>&1; rc=$?; tail -25 gpurun_out/bench_embed.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_embed -o run -- python scripts/bench_embed.py > gpurun_out/prof_embed.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py gpurun_out/prof_embed > gpurun_out/prof_embed_summary.txt 2>&1; head -25 gpurun_out/prof_embed_summary.txt
