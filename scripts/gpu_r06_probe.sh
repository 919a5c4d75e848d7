#!/bin/bash
# Round-6 kernel probes on one box: decode-GEMM lockstep ablation (abl 3 vs 131), prefill GEMM baseline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_dgemm.py --ablate --abl 0 3 131 129 1 0 3 131 129 1 --out gpurun_out/r06_dgemm_nobar.jsonl > gpurun_out/r06_dgemm_nobar.log 2>&1 || { tail -20 gpurun_out/r06_dgemm_nobar.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06_dgemm_nobar.jsonl"):
    r = json.loads(l); print(r["shape"], {k: v for k, v in r.items() if "abl" in k})
PY
timeout -k 10 400 python -u scripts/bench_pgemm.py --shapes qkv o gate_up down --variants packed --out gpurun_out/r06_pgemm_base.jsonl > gpurun_out/r06_pgemm_base.log 2>&1 || { tail -20 gpurun_out/r06_pgemm_base.log; exit 1; }
tail -4 gpurun_out/r06_pgemm_base.log
