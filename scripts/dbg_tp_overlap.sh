# TP=2 bench rehearsal on one GPU, ranks started directly (no torchrun) so each one's faulthandler
# dumps every thread's stack when its time limit sends SIGABRT: where does the overlapped prefill stall?
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29536 WORLD_SIZE=2 CFC_DIST_BACKEND=gloo PYTHONFAULTHANDLER=1
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -s ABRT -k 10 150 python -u bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 \
    --threads-per-gpu 32 --max-new 64 --latency-rate 0 --service-latency-rate 0 \
    > gpurun_out/tpdbg_$r.out 2> gpurun_out/tpdbg_$r.err &
done
wait
echo done
