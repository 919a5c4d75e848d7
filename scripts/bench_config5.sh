#!/bin/bash
# BASELINE config 5 on one MI355X: Llama-3-70B summarizer + 100M-vector HBM index, reduced steps
# (as profiles/r05_llama3_70b_100M_index_1gpu.log), with the topic-search probe over the 100M rows.
set -o pipefail
mkdir -p gpurun_out
cmd="python -u bench.py --model llama-3-70b --threads-per-gpu 32 --kv-max-prompt 3072 --index-prefill 100000000 --steps 2 --warmup 1 --latency-rate 0 --service-latency-rate 0 --search-queries 16"
echo "# $cmd" > gpurun_out/r06_70b.log
timeout -k 10 900 $cmd > gpurun_out/r06_70b.out 2> gpurun_out/r06_70b.err; rc=$?
grep -h "\[bench\]" gpurun_out/r06_70b.err >> gpurun_out/r06_70b.log; cat gpurun_out/r06_70b.out >> gpurun_out/r06_70b.log
tail -3 gpurun_out/r06_70b.err | cut -c1-300; tail -1 gpurun_out/r06_70b.out | cut -c1-400
exit $rc
