#!/bin/bash
# PMC passes over the prefill GEMM variants vs the library, then the node pipeline bench.
export TMPDIR=/tmp; mkdir -p gpurun_out; rm -rf gpurun_out/pmc_pg1 gpurun_out/pmc_pg2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_pg1 -o run -- python3 scripts/pmc_pgemm.py > gpurun_out/pmc_pg1.log 2>&1; rc=$?; tail -2 gpurun_out/pmc_pg1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_pg2 -o run -- python3 scripts/pmc_pgemm.py > gpurun_out/pmc_pg2.log 2>&1; rc=$?; tail -2 gpurun_out/pmc_pg2.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc_pg1 > gpurun_out/pmc_pgemm_summary.txt; python3 scripts/pmc_summary.py gpurun_out/pmc_pg2 >> gpurun_out/pmc_pgemm_summary.txt
find gpurun_out/pmc_pg1 gpurun_out/pmc_pg2 -name '*.csv' -size +2M -delete
cat gpurun_out/pmc_pgemm_summary.txt
timeout -k 10 400 python -u bench.py --pipeline node --steps 3 --warmup 1 > gpurun_out/bench_node.log 2>&1; rc=$?; tail -4 gpurun_out/bench_node.log; exit $rc
