#!/bin/bash
# Fused kNN scan: default loads vs nontemporal loads (100M x 384), A/B/A/B, plus numerics with nt on.
export TMPDIR=/tmp; mkdir -p gpurun_out
CFC_KNN_NT=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "knn" --timeout 200 --timeout-method thread > gpurun_out/pytest_knn_nt.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_knn_nt.log; [ $rc -eq 0 ] || exit $rc
for nt in 0 1 0 1; do
  CFC_KNN_NT=$nt timeout -k 10 300 python -u scripts/bench_knn.py 1e8 > gpurun_out/bench_knn_nt$nt.log 2>&1; rc=$?; echo "nt=$nt"; grep "^nq=" gpurun_out/bench_knn_nt$nt.log; [ $rc -eq 0 ] || exit $rc
done
