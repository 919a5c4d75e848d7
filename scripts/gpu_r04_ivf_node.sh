#!/bin/bash
# Round-4: pp GEMM W1-early probe on all four prefill shapes; IVF quality/speed on uniform and
# MiniLM-tiled data (10M rows, nprobe 8/32/128); the node pipeline (real services) vs bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/probe_pgemm_pp.py --probes pf1_g8 w1e_g8 --out gpurun_out/pgemm_w1e.jsonl > gpurun_out/pgemm_w1e.log 2>&1 || { tail -20 gpurun_out/pgemm_w1e.log; exit 1; }
grep shape gpurun_out/pgemm_w1e.log | cut -c1-400
timeout -k 10 500 python -u scripts/bench_ivf.py --n 1e7 --data uniform --out gpurun_out/ivf_r04.jsonl > gpurun_out/ivf_uniform.log 2>&1 || { tail -20 gpurun_out/ivf_uniform.log; exit 1; }
grep nprobe gpurun_out/ivf_uniform.log | cut -c1-300
timeout -k 10 600 python -u scripts/bench_ivf.py --n 1e7 --data minilm --unique 100000 --out gpurun_out/ivf_r04.jsonl > gpurun_out/ivf_minilm.log 2>&1 || { tail -20 gpurun_out/ivf_minilm.log; exit 1; }
grep nprobe gpurun_out/ivf_minilm.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "knn" > gpurun_out/knn_tests.log 2>&1 || { tail -30 gpurun_out/knn_tests.log; exit 1; }
tail -1 gpurun_out/knn_tests.log
timeout -k 10 400 python -u scripts/bench_knn.py 1e8 > gpurun_out/bench_knn_r04b.log 2>&1 || { tail -20 gpurun_out/bench_knn_r04b.log; exit 1; }
grep -E "^nq" gpurun_out/bench_knn_r04b.log
