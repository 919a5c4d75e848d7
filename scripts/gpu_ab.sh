#!/bin/bash
# build -> all GPU tests -> default bench -> llm-only A/B of an env toggle (e.g. CFC_FUSED_DECODE=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; grep "\[bench\] step\|metric" gpurun_out/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --llm-only --steps 2 --warmup 1 > gpurun_out/bench_llm_a.log 2>&1; rc=$?; grep "metric" gpurun_out/bench_llm_a.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 env "$@" python bench.py --llm-only --steps 2 --warmup 1 > gpurun_out/bench_llm_b.log 2>&1; rc=$?; grep "metric" gpurun_out/bench_llm_b.log | cut -c1-200; exit $rc
