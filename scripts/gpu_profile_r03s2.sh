#!/bin/bash
# Round-3 profiles: the headline bench (decode on the packed decode GEMM) and the encoder batch,
# rocprofv3 kernel-trace + stats; the encoder run writes BOTH csv (ns) and rocpd so the summary's
# unit handling of the SQLite path is checked against the csv.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/prof_embed
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps 1 --warmup 0 > gpurun_out/prof_bench.log 2>&1; rc=$?
tail -2 gpurun_out/prof_bench.log; [ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py gpurun_out/prof gpurun_out/prof_summary_s2.txt > /dev/null
find gpurun_out/prof -name '*kernel_trace.csv' -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d gpurun_out/prof_embed -o run -- \
  python scripts/bench_embed.py > gpurun_out/prof_embed.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/prof_embed.log; exit $rc; }
python scripts/prof_summary.py gpurun_out/prof_embed gpurun_out/prof_embed_summary_s2.txt > /dev/null
find gpurun_out/prof_embed -name '*kernel_trace.csv' -delete
head -30 gpurun_out/prof_summary_s2.txt
head -14 gpurun_out/prof_embed_summary_s2.txt
