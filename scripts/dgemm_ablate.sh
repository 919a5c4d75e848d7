#!/bin/bash
# Decode-GEMM ablation A/B in one process (scripts/bench_dgemm.py --ablate; ablation codes in
# csrc/kernels/dgemm.hip above dgemm_kernel).  Usage: scripts/dgemm_ablate.sh NAME ABL...
# writes gpurun_out/NAME.jsonl.  Round-6 calls (their jsonl files are in profiles/):
#   r06_dgemm_nobar  0 3 131 129 1 0 3 131 129 1   (per-stage workgroup barrier)
#   r06_dgemm_tail   0 256 3 259 0 256 3 259       (ring tail: straight-line peel, rejected)
#   r06_dgemm_tail2  0 256 3 259 0 256 3 259       (ring tail: out-of-range buffer loads)
#   r06_dgemm_xt     0 512 0 512 0 512             (W fragment as the MFMA A operand)
set -o pipefail
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 ${ABL_LIMIT:-400} python -u scripts/bench_dgemm.py --ablate --abl "$@" --out gpurun_out/$name.jsonl \
  > gpurun_out/$name.log 2>&1 || { tail -20 gpurun_out/$name.log; exit 1; }
python - "$name" <<'PY'
import json, sys
for l in open(f"gpurun_out/{sys.argv[1]}.jsonl"):
    r = json.loads(l)
    print(r["shape"], {k: v for k, v in r.items() if "abl" in k or k.startswith("pk_bn")})
PY
