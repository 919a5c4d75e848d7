#!/bin/bash
# lane-swap (v_permlane32/16_swap) reductions and SwiGLU epilogues: GPU suite, then the kernels they touch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/perm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/perm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/bench_attn.py > gpurun_out/perm_attn.log 2>&1 || { tail -5 gpurun_out/perm_attn.log; exit 1; }
cat gpurun_out/perm_attn.log | grep -v amdgpu.ids
timeout -k 10 400 python3 scripts/probe_pgemm_k.py gpurun_out/pgemm_k4.jsonl pps,ppp > gpurun_out/pgemm_k4.log 2>&1 || { tail -5 gpurun_out/pgemm_k4.log; exit 1; }
grep fit gpurun_out/pgemm_k4.log
timeout -k 10 300 python -u scripts/bench_dgemm.py --out gpurun_out/perm_dgemm.jsonl > gpurun_out/perm_dgemm.log 2>&1 || { tail -5 gpurun_out/perm_dgemm.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/perm_dgemm.jsonl"):
    r = json.loads(l)
    if r.get("M") == 128: print(r["shape"], {k: v for k, v in r.items() if k.endswith("_us") and ("pk" in k or "lib" in k)})
PY
