# rocprofv3 per-kernel durations of scripts/probe_dgemm_srr.py for several (bn, split) choices of
# the o and down projections; keeps each run's kernel stats under gpurun_out/dgemm_srr/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dgemm_srr
for cfg in "down 128 8" "down 64 4" "down 128 7" "down 64 8" "o 64 4" "o 128 8" "o 64 2" "o 128 4"; do
  tag=$(echo $cfg | tr ' ' _)
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ds_$tag -o run -- \
    python3 $R/scripts/probe_dgemm_srr.py $cfg > $R/gpurun_out/dgemm_srr/$tag.log 2>&1 || exit 1
  cp "$(find /tmp/ds_$tag -name '*kernel_stats.csv' | head -1)" $R/gpurun_out/dgemm_srr/$tag.kernel_stats.csv
  rm -rf /tmp/ds_$tag
done
