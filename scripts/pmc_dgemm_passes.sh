#!/bin/bash
# PMC passes (kernel-trace counters only, one pass per counter set, each under its own KILL timeout)
# of the decode GEMM at M = 128, full kernel (abl 0) vs no X DMA (abl 1): where does the X stream cost?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE"
for shape in gate_up down; do
  for abl in 0 1; do
    i=0
    for P in "$P1" "$P2" "$P3"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d /tmp/pmc_${shape}_${abl}_$i -o run -- \
        python3 $R/scripts/pmc_dgemm_abl.py $shape $abl > $R/gpurun_out/pmc/${shape}_${abl}_$i.log 2>&1 || { echo "pass $shape $abl $i failed"; tail -5 $R/gpurun_out/pmc/${shape}_${abl}_$i.log; exit 1; }
      f=$(find /tmp/pmc_${shape}_${abl}_$i -name '*counter_collection.csv' | head -1)
      grep -i "dgemm_kernel" "$f" > $R/gpurun_out/pmc/${shape}_${abl}_$i.csv; head -1 "$f" > $R/gpurun_out/pmc/header.csv
      rm -rf /tmp/pmc_${shape}_${abl}_$i
    done
  done
done
echo pmc done
