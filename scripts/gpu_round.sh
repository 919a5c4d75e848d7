#!/bin/bash
# One GPU session: kernel numerics -> engine tests -> smoke -> small bench -> full bench.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_kernels.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --llm-only --threads-per-gpu 16 --max-new 64 --steps 1 --warmup 1 > gpurun_out/bench_small.log 2>&1; rc=$?; tail -4 gpurun_out/bench_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --llm-only "$@" > gpurun_out/bench_llm.log 2>&1; rc=$?; tail -6 gpurun_out/bench_llm.log; exit $rc
