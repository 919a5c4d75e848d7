#!/bin/bash
# Round-6 first GPU call: decode-GEMM baseline on this box, then the overlapped-TP-prefill stall
# rehearsal with the one-shot all-reduce's error counter and epochs printed per rank.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_dgemm.py --out gpurun_out/r06_dgemm_base.jsonl > gpurun_out/r06_dgemm_base.log 2>&1 || { tail -20 gpurun_out/r06_dgemm_base.log; exit 1; }
tail -8 gpurun_out/r06_dgemm_base.log
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29536 WORLD_SIZE=2 CFC_DIST_BACKEND=gloo PYTHONFAULTHANDLER=1
export CFC_TP_PREFILL_OVERLAP=force CFC_AR_DEBUG=1
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -s ABRT -k 10 170 python -u bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 \
    --threads-per-gpu 32 --max-new 64 --latency-rate 0 --service-latency-rate 0 \
    > gpurun_out/r06_tpdbg_$r.out 2> gpurun_out/r06_tpdbg_$r.err &
done
wait
grep -h "ar-debug\|\[bench\]" gpurun_out/r06_tpdbg_0.out gpurun_out/r06_tpdbg_0.err gpurun_out/r06_tpdbg_1.out | head -40
