#!/bin/bash
# BASELINE config 5 retrieval half at full scale: 100M x 384 bf16 flat (fused scan + top-k), then IVF-flat.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_knn.py 1e8 > gpurun_out/bench_knn_100M.log 2>&1; rc=$?; tail -5 gpurun_out/bench_knn_100M.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u scripts/bench_knn.py 1e8 --ivf 10000 32 > gpurun_out/bench_ivf_100M.log 2>&1; rc=$?; tail -6 gpurun_out/bench_ivf_100M.log | cut -c1-500; exit $rc
