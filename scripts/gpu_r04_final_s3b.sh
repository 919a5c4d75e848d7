#!/bin/bash
# Round-4 final validation on one box: every GPU test, smoke, the headline bench (5 steps) and the
# node pipeline (4 steps) back to back, then a clean headline profile (no latency probe).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final_s3b.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_final_s3b.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final_s3b.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final_s3b.log 2>&1 || { tail -30 gpurun_out/smoke_final_s3b.log; exit 1; }
tail -1 gpurun_out/smoke_final_s3b.log
timeout -k 10 700 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_final_s3b.log 2>&1 || { tail -30 gpurun_out/bench_final_s3b.log; exit 1; }
grep -E '^\[bench\] step|"metric"' gpurun_out/bench_final_s3b.log | cut -c1-600
timeout -k 10 600 python -u bench.py --pipeline node --steps 4 --warmup 1 > gpurun_out/node_final_s3b.log 2>&1 || { tail -30 gpurun_out/node_final_s3b.log; exit 1; }
grep -E 'step [0-9]|"metric"' gpurun_out/node_final_s3b.log | cut -c1-400
