#!/bin/bash
# Decode GEMM: the no-reload ring tail (abl 0 / 3) against the round-5 re-reading tail (abl 256 / 259),
# A/B/A/B in one process; the decode-GEMM GPU tests; then the TP tests with the fused fp32
# all-reduce + residual + RMSNorm (one-shot IPC kernel).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_dgemm.py --ablate --abl 0 256 3 259 0 256 3 259 --out gpurun_out/r06_dgemm_tail.jsonl > gpurun_out/r06_dgemm_tail.log 2>&1 || { tail -20 gpurun_out/r06_dgemm_tail.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06_dgemm_tail.jsonl"):
    r = json.loads(l); print(r["shape"], {k: v for k, v in r.items() if "abl" in k or k.startswith("pk_bn") or "err_packed" in k})
PY
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dgemm" --timeout 300 --timeout-method thread > gpurun_out/r06_dgemm_tests.log 2>&1 || { tail -30 gpurun_out/r06_dgemm_tests.log; exit 1; }
tail -2 gpurun_out/r06_dgemm_tests.log
timeout -k 10 1500 python -u -m pytest tests/test_custom_ar_gpu.py -x -v --timeout 900 --timeout-method thread > gpurun_out/r06_custom_ar_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|sigma" gpurun_out/r06_custom_ar_tests.log | tail -20; exit $rc
