#!/bin/bash
# PMC pass over the decode GEMM shapes: HBM bytes (FETCH_SIZE) and matrix-pipe / wave activity.
export TMPDIR=/tmp; mkdir -p gpurun_out; rm -rf gpurun_out/pmc_dg
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_dg -o run -- python3 scripts/pmc_dgemm.py > gpurun_out/pmc_dg.log 2>&1; rc=$?; tail -6 gpurun_out/pmc_dg.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc_dg > gpurun_out/pmc_dgemm_summary.txt
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/pmc_dg/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "dgemm_kernel" in r.get("Kernel_Name", ""):
            rows.append((r["Kernel_Name"].split("(")[0][-40:], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
with open("gpurun_out/pmc_dgemm_summary.txt", "a") as fh:
    fh.write("\n# per-dispatch kernel time (us) under the PMC pass\n")
    for k, t in rows:
        fh.write(f"{k} {t:.1f}\n")
PY
find gpurun_out/pmc_dg -name '*.csv' -size +2M -delete
cat gpurun_out/pmc_dgemm_summary.txt | grep -v "^\s*$" | head -60
