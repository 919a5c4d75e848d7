#!/bin/bash
# Decode GEMM with a 12-stage W register ring at BM = 128 (was 8): tests, then timing at M = 128.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "dgemm" > gpurun_out/dgd12_tests.log 2>&1 || { tail -30 gpurun_out/dgd12_tests.log; exit 1; }
tail -1 gpurun_out/dgd12_tests.log
timeout -k 10 500 python -u scripts/bench_dgemm.py --m 128 --shapes qkv o gate_up down --ablate --abl 0 3 0 3 --out gpurun_out/dgd12.jsonl > gpurun_out/dgd12.log 2>&1 || { tail -20 gpurun_out/dgd12.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/dgd12.jsonl"):
    d = json.loads(l)
    print(d["shape"], d["config"], {k: v for k, v in d.items() if k.startswith("pk_abl") or k.endswith("swiglu_us")})
PY
