#!/bin/bash
# Interleaved A/B of two builds of libcfc_kernels.so (build/ab/old.so vs build/ab/new.so) on any
# python command, on one box; restores new.so at the end.
#   scripts/ab_lib.sh [ROUNDS=3] -- python scripts/bench_attn.py ...
# build/ab is listed in .gpurunignore: drop that line for the call that runs this script.  (The
# round-5 ab_kernel_lib / ab_kernel_lib_embed runs: bench_attn prefill cases, bench_embed.)
set -o pipefail
ROUNDS=${1:-3}; shift; [ "$1" = "--" ] && shift
mkdir -p gpurun_out
LIB=copilot_for_consensus_amd/_lib/libcfc_kernels.so
for r in $(seq 1 "$ROUNDS"); do
  for v in old new; do
    cp build/ab/$v.so $LIB
    echo "== $v" >> gpurun_out/ab_lib.log
    timeout -k 10 300 "$@" >> gpurun_out/ab_lib.log 2>&1 || { cp build/ab/new.so $LIB; exit 1; }
  done
done
cp build/ab/new.so $LIB
cat gpurun_out/ab_lib.log
