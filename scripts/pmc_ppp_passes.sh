#!/bin/bash
# PMC passes (kernel-trace counters only, one pass per counter set under its own KILL timeout) of
# the prefill GEMM: persistent vs one-tile ping-pong vs library at qkv / gate_up, per-kernel means.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_ppp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/pmc_ppp_$i -o run -- \
    python3 $R/scripts/pmc_ppp.py > $R/gpurun_out/pmc_ppp/pass_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc_ppp/pass_$i.log; exit 1; }
  f=$(find /tmp/pmc_ppp_$i -name '*counter_collection.csv' | head -1)
  cp "$f" $R/gpurun_out/pmc_ppp/pass_$i.csv
  rm -rf /tmp/pmc_ppp_$i
done
echo pmc done
