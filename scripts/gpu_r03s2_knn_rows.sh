#!/bin/bash
# Flat kNN with per-query-count chunk rows: numerics, then the 100M x 384 scan at nq 1 / 16.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_vectorstore_contract.py -x -q -k "knn or ivf or flat or vector" --timeout 200 --timeout-method thread > gpurun_out/pytest_knn.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_knn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_knn.py 1e8 > gpurun_out/bench_knn_100M_rows.log 2>&1; rc=$?; tail -4 gpurun_out/bench_knn_100M_rows.log | cut -c1-300; exit $rc
