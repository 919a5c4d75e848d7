cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe -o run -- python3 $R/scripts/bench_embed.py > $R/gpurun_out/prof_embed.log 2>&1 || exit 1
cp "$(find /tmp/pe -name '*kernel_stats.csv' | head -1)" $R/gpurun_out/prof_embed_kernel_stats.csv
