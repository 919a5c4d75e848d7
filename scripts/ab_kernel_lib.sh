#!/bin/bash
# A/B of two builds of libcfc_kernels.so (build/ab/old.so vs build/ab/new.so) on the prefill
# attention micro-benchmark, interleaved; restores new.so at the end.  build/ab is listed in
# .gpurunignore (20 MB per call otherwise): drop that line for the call that runs this script.
set -o pipefail
mkdir -p gpurun_out
LIB=copilot_for_consensus_amd/_lib/libcfc_kernels.so
for v in old new old new old new; do
  cp build/ab/$v.so $LIB
  echo "== $v" >> gpurun_out/ab_kernel_lib.log
  timeout -k 10 120 python -c "
import sys; sys.path.insert(0, 'scripts'); import bench_attn
bench_attn.prefill_case(iters=20); bench_attn.prefill_case(nseq=1, L=16384, iters=5)" >> gpurun_out/ab_kernel_lib.log 2>&1 || exit 1
done
cp build/ab/new.so $LIB
cat gpurun_out/ab_kernel_lib.log
