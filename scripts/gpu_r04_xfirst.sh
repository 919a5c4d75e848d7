#!/bin/bash
# dgemm X-first probe, repeated A/B/A/B/A/B on every decode shape (M = 128).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/bench_dgemm.py --ablate --abl 0 16 0 16 0 16 --calls 128 --out gpurun_out/dgemm_xfirst2.jsonl > gpurun_out/dgemm_xfirst2.log 2>&1 || { tail -20 gpurun_out/dgemm_xfirst2.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/dgemm_xfirst2.jsonl"):
    d = json.loads(l)
    print(d["shape"], {k: v for k, v in d.items() if k.startswith("pk_abl")})
PY
