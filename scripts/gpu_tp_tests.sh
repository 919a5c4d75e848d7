#!/bin/bash
# TP GPU tests after the fp32 row-parallel sums: Llama-3-70B TP=2 against TP=1 (with TP=1's own
# decode as the floor) and the TP=4 / TP=8 one-shot tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_custom_ar_gpu.py -v -s --timeout 900 --timeout-method thread -k "70b or wide" > gpurun_out/r06_tp_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|sigma" gpurun_out/r06_tp_tests.log | tail -20; exit $rc
