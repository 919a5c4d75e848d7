#!/bin/bash
# Decode GEMM ablations at M = 128 (timing probes, wrong results by construction): 1 no X loads,
# 2 no MFMA, 3 neither, 8 temporal W loads -- what bounds each projection.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/bench_dgemm.py --m 128 --shapes qkv o gate_up down --ablate --abl 0 1 2 3 8 --out gpurun_out/dgabl.jsonl > gpurun_out/dgabl.log 2>&1 || { tail -20 gpurun_out/dgabl.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/dgabl.jsonl"):
    d = json.loads(l)
    print(d["shape"], d["config"], d["w_MB"], {k: v for k, v in d.items() if k.startswith("pk_abl")})
PY
