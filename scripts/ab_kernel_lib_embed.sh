#!/bin/bash
# A/B of two builds of libcfc_kernels.so (build/ab/old.so vs new.so) on the encoder benchmark
# (scripts/bench_embed.py: MiniLM-L6 and bge-small, batch 256), interleaved; restores new.so.
# build/ab is listed in .gpurunignore: drop that line for the call that runs this script.
set -o pipefail
mkdir -p gpurun_out
LIB=copilot_for_consensus_amd/_lib/libcfc_kernels.so
for v in old new old new; do
  cp build/ab/$v.so $LIB
  echo "== $v" >> gpurun_out/ab_kernel_lib_embed.log
  timeout -k 10 300 python scripts/bench_embed.py 2>/dev/null | grep '^{' >> gpurun_out/ab_kernel_lib_embed.log || exit 1
done
cp build/ab/new.so $LIB
