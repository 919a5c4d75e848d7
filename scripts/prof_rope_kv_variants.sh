# rocprofv3 per-kernel durations of each probe_rope_kv_step.py variant (one process per variant);
# keeps only the kernel stats table of each run under gpurun_out/rope_prof/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rope_prof
for v in part part_noKV part_vwt bf16 bf16_noV; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp_$v -o run -- python3 $R/scripts/probe_rope_kv_step.py $v > $R/gpurun_out/rope_prof/$v.log 2>&1 || exit 1
  f=$(find /tmp/rp_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $R/gpurun_out/rope_prof/$v.kernel_stats.csv
  du -sh /tmp/rp_$v >> $R/gpurun_out/rope_prof/$v.log
  rm -rf /tmp/rp_$v
done
