#!/bin/bash
# DP=2 services topology on one GPU (gloo control plane, both ranks on the card): the light-load
# service latency (archive submit -> report stored, 0.5 threads/s) with the control plane's waits as
# blocking TCPStore waits (round 6) vs round 5's 1-20 ms check polling (CFC_DP_WAIT=poll).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in poll block; do
  CFC_NODE_MIN_ADMIT=1 CFC_NODE_ADMIT_WAIT_MS=50 CFC_DP_WAIT=$mode CFC_DIST_BACKEND=gloo timeout -k 10 520 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 2953${#mode} bench.py --gpus 2 --pipeline node --steps 1 --warmup 1 \
    --threads-per-gpu 64 --service-latency-rate 0.5 --service-latency-threads 12 \
    > gpurun_out/r06_dpwait_$mode.out 2> gpurun_out/r06_dpwait_$mode.err || { tail -5 gpurun_out/r06_dpwait_$mode.err; exit 1; }
  python - $mode <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r06_dpwait_{sys.argv[1]}.out").read().strip().splitlines()[-1])
print(sys.argv[1], "value", d["value"], "p50", d["p50_summary_latency_s"], "light", d["latency_service_light"]["p50_s"], d["latency_service_light"]["p95_s"])
PY
done
