#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/bench_dgemm.py --m 128 --shapes qkv o down --split-sweep --out gpurun_out/dgsweep.jsonl > gpurun_out/dgsweep.log 2>&1 || { tail -20 gpurun_out/dgsweep.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/dgsweep.jsonl"):
    d = json.loads(l)
    pk = sorted((v, k) for k, v in d.items() if k.startswith("pk_bn"))
    print(d["shape"], d["config"], pk[:6])
PY
