#!/bin/bash
# Round-4 A/B on one box: headline bench (no latency probe) with the round-4 defaults vs the
# library prefill GEMM (both weight copies) vs the unfused RoPE/KV write; decode-GEMM X-first probe;
# large-k flat kNN (tests + 100M bench).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > gpurun_out/ab_$name.log 2>&1 || { tail -20 gpurun_out/ab_$name.log; return 1; }
  grep -E '^\[bench\] step|"metric"' gpurun_out/ab_$name.log | cut -c1-330
}
run default && \
run libprefill CFC_WEIGHTS_PACKED_ONLY=0 CFC_PREFILL_GEMM=lib && \
run unfusedrope CFC_DECODE_ROPE_FUSED=0 && \
timeout -k 10 300 python -u scripts/bench_dgemm.py --ablate --abl 0 16 --out gpurun_out/dgemm_xfirst.jsonl > gpurun_out/dgemm_xfirst.log 2>&1 && \
grep -o '"shape[^,]*\|"pk_abl[^,]*' gpurun_out/dgemm_xfirst.log | paste -sd' ' && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "knn" > gpurun_out/knn_tests.log 2>&1 && tail -2 gpurun_out/knn_tests.log && \
timeout -k 10 400 python -u scripts/bench_knn.py 1e8 > gpurun_out/bench_knn_r04.log 2>&1 && grep -E "^nq" gpurun_out/bench_knn_r04.log
