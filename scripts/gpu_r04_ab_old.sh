#!/bin/bash
# Headline A/B on one box: the session-start build (_old worktree, commit 020879a) vs now.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
root=$(pwd)
(cd _old && timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > $root/gpurun_out/ab_old.log 2>&1) || { tail -30 gpurun_out/ab_old.log; exit 1; }
echo "== old"; grep -E '^\[bench\] step' gpurun_out/ab_old.log | cut -c1-260
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > gpurun_out/ab_new.log 2>&1 || { tail -30 gpurun_out/ab_new.log; exit 1; }
echo "== new"; grep -E '^\[bench\] step' gpurun_out/ab_new.log | cut -c1-260
