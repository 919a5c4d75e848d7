#!/bin/bash
# build -> all GPU tests -> full bench (A) -> full bench with an env toggle (B) -> attention microbench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_a.log 2>&1; rc=$?; grep "\[bench\] step\|metric" gpurun_out/bench_a.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 env "$@" python bench.py --steps 3 --warmup 1 > gpurun_out/bench_b.log 2>&1; rc=$?; grep "\[bench\] step\|metric" gpurun_out/bench_b.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_attn.py > gpurun_out/bench_attn.log 2>&1; rc=$?; cat gpurun_out/bench_attn.log | grep -v amdgpu.ids; exit $rc
