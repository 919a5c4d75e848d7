#!/bin/bash
# build -> all GPU tests -> smoke -> headline bench -> config benches (embedding, 100M kNN)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1; rc=$?; grep "\[bench\] step\|metric" gpurun_out/bench.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_embed.py > gpurun_out/bench_embed.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/bench_embed.log; exit $rc
