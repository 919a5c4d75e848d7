#!/bin/bash
# LDS-staged epilogue: bit-identity / numerics GPU tests, then pp vs pps (packed weights) vs the library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "pgemm" > gpurun_out/pps_tests.log 2>&1 || { tail -30 gpurun_out/pps_tests.log; exit 1; }
tail -1 gpurun_out/pps_tests.log
timeout -k 10 500 python -u scripts/bench_pgemm.py --shapes qkv o gate_up down --variants packed packed_pps --out gpurun_out/pgemm_pps.jsonl > gpurun_out/pgemm_pps.log 2>&1 || { tail -20 gpurun_out/pgemm_pps.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/pgemm_pps.jsonl"):
    d = json.loads(l)
    print(d["shape"], {k: d[k] for k in d if k.endswith("_TFs") or k.startswith("maxdiff") or k.startswith("err_")})
PY
