#!/bin/bash
# Round-5 evidence on one GPU: rocprofv3 of one headline batch, the headline as the driver runs it
# (20 timed steps + 5 warm-up), and the services.main DP topology as 2 ranks sharing the GPU (gloo).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_profile.sh --steps 1 --warmup 0 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 || exit $?
cp gpurun_out/prof_summary.txt gpurun_out/r05_prof_full_bench.txt
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_20steps.out 2> gpurun_out/r05_bench_20steps.err || exit $?
tail -1 gpurun_out/r05_bench_20steps.out
CFC_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --pipeline node --steps 2 --warmup 1 \
  > gpurun_out/r05_node_dp2_1gpu.out 2> gpurun_out/r05_node_dp2_1gpu.err || exit $?
tail -1 gpurun_out/r05_node_dp2_1gpu.out
