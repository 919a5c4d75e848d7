#!/bin/bash
# Decode GEMM with the W fragment as the MFMA A operand (16-byte epilogue stores, abl 0) vs the
# round-5 orientation (abl 512), A/B/A/B in one process; decode-GEMM + TP GPU tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_dgemm.py --ablate --abl 0 512 0 512 0 512 --out gpurun_out/r06_dgemm_xt.jsonl > gpurun_out/r06_dgemm_xt.log 2>&1 || { tail -20 gpurun_out/r06_dgemm_xt.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06_dgemm_xt.jsonl"):
    r = json.loads(l); print(r["shape"], {k: v for k, v in r.items() if "abl" in k or k.startswith("pk_") or k.startswith("err")})
PY
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_xt_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06_xt_tests.log; exit $rc
