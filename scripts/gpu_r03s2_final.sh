#!/bin/bash
# End-of-session check of HEAD: every GPU test, smoke, the 100M kNN bench, the headline bench.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_knn.py 1e8 > gpurun_out/bench_knn_100M_final.log 2>&1; rc=$?; grep "^nq=" gpurun_out/bench_knn_100M_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
