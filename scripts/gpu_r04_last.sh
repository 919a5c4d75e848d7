#!/bin/bash
# Last check of the session: every GPU test and smoke at HEAD.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_last.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_last.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_last.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1 || { tail -30 gpurun_out/smoke_last.log; exit 1; }
tail -1 gpurun_out/smoke_last.log
