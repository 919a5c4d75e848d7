#!/bin/bash
# FETCH_SIZE of the decode attention kernel (one PMC pass, kernel-trace counters only)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_dec
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc_dec -o run -- \
  python3 $R/scripts/pmc_decode_attn.py > $R/gpurun_out/pmc_dec/run.log 2>&1 || { tail -5 $R/gpurun_out/pmc_dec/run.log; exit 1; }
cp $(find /tmp/pmc_dec -name '*counter_collection.csv' | head -1) $R/gpurun_out/pmc_dec/counters.csv
cp $(find /tmp/pmc_dec -name '*kernel_trace.csv' | head -1) $R/gpurun_out/pmc_dec/trace.csv 2>/dev/null
rm -rf /tmp/pmc_dec
grep "kv bytes" $R/gpurun_out/pmc_dec/run.log
echo done
