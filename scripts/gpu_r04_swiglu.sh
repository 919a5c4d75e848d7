#!/bin/bash
# SwiGLU epilogue over both lane halves: pgemm tests (numerics, variant bit-identity), gate_up timing.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -x --timeout 120 --timeout-method thread -k "pgemm or prefill" > gpurun_out/swiglu_rcp_tests.log 2>&1 || { tail -30 gpurun_out/swiglu_rcp_tests.log; exit 1; }
tail -1 gpurun_out/swiglu_rcp_tests.log
timeout -k 10 300 python -u scripts/bench_pgemm.py --shapes gate_up qkv --variants packed packed_pps --out gpurun_out/pgemm_swiglu_rcp.jsonl > gpurun_out/pgemm_swiglu_rcp.log 2>&1 || { tail -20 gpurun_out/pgemm_swiglu_rcp.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/pgemm_swiglu_rcp.jsonl"):
    d = json.loads(l)
    print(d["shape"], {k: d[k] for k in d if k.endswith("_TFs") or k.startswith("maxdiff") or k.startswith("err_")})
PY
