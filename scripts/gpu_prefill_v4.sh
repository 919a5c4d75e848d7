#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
for v in 2 3; do
  CFC_PREFILL_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k prefill > gpurun_out/pytest_pf_v$v.log 2>&1; rc=$?; echo "variant $v tests:"; tail -3 gpurun_out/pytest_pf_v$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 2 3; do
  echo "variant $v:"; CFC_PREFILL_VARIANT=$v timeout -k 10 200 python scripts/bench_attn.py 2>&1 | grep prefill || exit 1
done
CFC_PREFILL_VARIANT=2 timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -x -q 2>&1 | tail -2
