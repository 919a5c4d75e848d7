#!/bin/bash
# Decode GEMM: out-of-range tail refills (abl 0 / 3) vs the round-5 re-reading tail (abl 256 / 259),
# A/B/A/B in one process; decode / prefill GEMM GPU tests; the TP tests (fp32 row-parallel sums).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_dgemm.py --ablate --abl 0 256 3 259 0 256 3 259 --out gpurun_out/r06_dgemm_tail2.jsonl > gpurun_out/r06_dgemm_tail2.log 2>&1 || { tail -20 gpurun_out/r06_dgemm_tail2.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06_dgemm_tail2.jsonl"):
    r = json.loads(l); print(r["shape"], {k: v for k, v in r.items() if "abl" in k or k.startswith("pk_bn")})
PY
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "dgemm or pgemm" --timeout 300 --timeout-method thread > gpurun_out/r06_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r06_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r06_gemm_tests.log
timeout -k 10 1000 python -u -m pytest tests/test_custom_ar_gpu.py -x -v --timeout 900 --timeout-method thread > gpurun_out/r06_custom_ar_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|sigma" gpurun_out/r06_custom_ar_tests.log | tail -20; exit $rc
