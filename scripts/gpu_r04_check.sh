#!/bin/bash
# Round-4 end-to-end check on the GPU: every GPU test, smoke(), and a short headline bench run.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_r04.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r04.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.log 2>&1 || { tail -30 gpurun_out/smoke_r04.log; exit 1; }
tail -2 gpurun_out/smoke_r04.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_r04.log 2>&1 || { tail -30 gpurun_out/bench_r04.log; exit 1; }
tail -8 gpurun_out/bench_r04.log
