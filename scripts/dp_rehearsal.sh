#!/bin/bash
# DP bench rehearsal on one GPU: the driver's multi-GPU command shape (one process per rank, env://
# rendezvous on 127.0.0.1) with WORLD_SIZE ranks sharing the card over a gloo process group, reduced
# steps / threads.  DP=${DP:-2}; extra bench flags via BENCH_ARGS.
set -o pipefail
mkdir -p gpurun_out
DP=${DP:-2}
export MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29537} WORLD_SIZE=$DP CFC_DIST_BACKEND=gloo PYTHONFAULTHANDLER=1
pids=()
for ((r = 0; r < DP; r++)); do
  RANK=$r LOCAL_RANK=$r timeout -s ABRT -k 10 ${DP_LIMIT:-300} python -u bench.py --gpus $DP --steps 2 --warmup 1 \
    --threads-per-gpu 32 --max-new 64 ${BENCH_ARGS} \
    > gpurun_out/dp_rehearsal_$r.out 2> gpurun_out/dp_rehearsal_$r.err &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep -h "\[bench\]" gpurun_out/dp_rehearsal_0.err | tail -4
tail -1 gpurun_out/dp_rehearsal_0.out
exit $rc
