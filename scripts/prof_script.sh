#!/bin/bash
# rocprofv3 kernel durations of one python script run (kernel trace + stats only; never PMC with
# trace domains), keeping the stats table as gpurun_out/prof_<TAG>.kernel_stats.csv.
#   scripts/prof_script.sh TAG scripts/probe_rope_kv_step.py part      (round-5 prof_rope_kv_variants)
#   scripts/prof_script.sh embed scripts/bench_embed.py                 (round-5 prof_embed)
#   scripts/prof_script.sh srr_down scripts/probe_dgemm_srr.py down 128 8   (round-5 prof_dgemm_srr)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
SCRIPT=$1; shift
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ps_$TAG -o run -- \
  python3 $R/$SCRIPT "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 1
cp "$(find /tmp/ps_$TAG -name '*kernel_stats.csv' | head -1)" $R/gpurun_out/prof_$TAG.kernel_stats.csv
rm -rf /tmp/ps_$TAG
