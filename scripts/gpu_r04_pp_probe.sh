#!/bin/bash
# Ping-pong prefill GEMM: probe timing (priority schemes, tile-order group) + PMC passes vs the library.
export TMPDIR=/tmp; mkdir -p gpurun_out; rm -rf gpurun_out/pmc_pp1 gpurun_out/pmc_pp2
timeout -k 10 300 python -u scripts/probe_pgemm_pp.py --out gpurun_out/pgemm_probe.jsonl > gpurun_out/probe_pp.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_pp1 -o run -- python3 scripts/probe_pgemm_pp.py --pmc qkv --probes pf0_g8 > gpurun_out/pmc_pp1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_pp2 -o run -- python3 scripts/probe_pgemm_pp.py --pmc qkv --probes pf0_g8 > gpurun_out/pmc_pp2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_pp1 > gpurun_out/pmc_pp_summary.txt; python3 scripts/pmc_summary.py gpurun_out/pmc_pp2 >> gpurun_out/pmc_pp_summary.txt
find gpurun_out/pmc_pp1 gpurun_out/pmc_pp2 -name '*.csv' -size +2M -delete
