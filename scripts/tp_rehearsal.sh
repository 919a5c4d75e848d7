#!/bin/bash
# TP=2 bench rehearsal on one GPU (gloo process group, both ranks on the card, the one-shot IPC
# all-reduce between them), ranks started directly so each one's faulthandler dumps every thread's
# stack if its time limit fires.  Environment passes through, e.g.
#   CFC_TP_PREFILL_OVERLAP=1 CFC_AR_DEBUG=1 scripts/tp_rehearsal.sh       (profiles/r06_tp2_overlap_gloo_1gpu.log)
set -o pipefail
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29536} WORLD_SIZE=2 CFC_DIST_BACKEND=gloo PYTHONFAULTHANDLER=1
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -s ABRT -k 10 ${TP_LIMIT:-240} python -u bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 \
    --threads-per-gpu 32 --max-new 64 --latency-rate 0 --service-latency-rate 0 --search-queries 0 \
    > gpurun_out/tp_rehearsal_$r.out 2> gpurun_out/tp_rehearsal_$r.err &
done
wait
grep -h "ar-debug\|\[bench\]" gpurun_out/tp_rehearsal_0.out gpurun_out/tp_rehearsal_0.err gpurun_out/tp_rehearsal_1.out
tail -1 gpurun_out/tp_rehearsal_0.out
