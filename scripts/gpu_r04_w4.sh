#!/bin/bash
# 4-wave and ping-pong prefill GEMMs: numerics tests, then timing vs the library on the headline shapes.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pgemm" > gpurun_out/t_pgemm_w4.log 2>&1 || { tail -30 gpurun_out/t_pgemm_w4.log; exit 1; }
tail -2 gpurun_out/t_pgemm_w4.log
timeout -k 10 400 python -u scripts/bench_pgemm.py --shapes qkv o gate_up down --variants stage2 packed packed_w4 w4 --out gpurun_out/pgemm_w4.jsonl > gpurun_out/b_pgemm_w4.log 2>&1 || exit $?
cat gpurun_out/b_pgemm_w4.log | grep shape | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.endswith('TFs')})"
