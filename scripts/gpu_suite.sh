#!/bin/bash
# The whole GPU test suite + smoke on one box (as the driver runs them at round end).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r06_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r06_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r06_smoke.log; exit $rc
