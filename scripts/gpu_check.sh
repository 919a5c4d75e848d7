#!/bin/bash
# GPU check of the in-tree build (extensions built on the CPU container beforehand):
# all GPU tests -> smoke -> end-to-end bench.  Each GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py "$@" > gpurun_out/bench.log 2>&1; rc=$?; tail -6 gpurun_out/bench.log; exit $rc
