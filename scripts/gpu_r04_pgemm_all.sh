#!/bin/bash
# Prefill GEMM round 4: numerics (pp / w4 / packed / packed GEMV), timing vs the library on the
# headline shapes, the ping-pong probes, and two PMC passes.  Every GPU step under its own timeout.
export TMPDIR=/tmp; mkdir -p gpurun_out; rm -rf gpurun_out/pmc_pp1 gpurun_out/pmc_pp2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pgemm or gemv_packed" > gpurun_out/t_pgemm_all.log 2>&1 || { tail -40 gpurun_out/t_pgemm_all.log; exit 1; }
tail -2 gpurun_out/t_pgemm_all.log
timeout -k 10 400 python -u scripts/bench_pgemm.py --shapes qkv o gate_up down --variants stage2 packed packed_w4 --out gpurun_out/pgemm_r04.jsonl > gpurun_out/b_pgemm_r04.log 2>&1 || { tail -20 gpurun_out/b_pgemm_r04.log; exit 1; }
grep shape gpurun_out/b_pgemm_r04.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if k.endswith('TFs') or k.startswith('err')})"
timeout -k 10 300 python -u scripts/probe_pgemm_pp.py --out gpurun_out/pgemm_probe.jsonl > gpurun_out/probe_pp.log 2>&1 || { tail -20 gpurun_out/probe_pp.log; exit 1; }
cat gpurun_out/probe_pp.log | grep shape
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_pp1 -o run -- python3 scripts/probe_pgemm_pp.py --pmc qkv --probes pf0_g8 > gpurun_out/pmc_pp1.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_pp1 > gpurun_out/pmc_pp_summary.txt
find gpurun_out/pmc_pp1 -name '*.csv' -size +2M -delete
grep -A9 "pgemm_pp\|Cijk" gpurun_out/pmc_pp_summary.txt | head -40
