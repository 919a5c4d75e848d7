#!/bin/bash
# 2 DP ranks on the one GPU of the box (gloo between them, both on cuda:0): the sharded-index data
# plane of the bench end to end with real models; then the 1-GPU headline bench for regression.
export TMPDIR=/tmp; mkdir -p gpurun_out
CFC_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --threads-per-gpu 32 --max-new 64 > gpurun_out/dp2_sharded_rehearsal.log 2>&1; rc=$?; tail -3 gpurun_out/dp2_sharded_rehearsal.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; tail -2 gpurun_out/bench.log | cut -c1-300; exit $rc
