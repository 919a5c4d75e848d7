#!/bin/bash
# Round-4 (d): shared-prefix KV blocks read through the caches in decode attention -- kernel test,
# then the headline A/B (CFC_DECODE_SHARED_CACHED=1 default vs 0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "paged_decode" > gpurun_out/d_tests.log 2>&1 || { tail -30 gpurun_out/d_tests.log; exit 1; }
tail -1 gpurun_out/d_tests.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --latency-rate 0 > gpurun_out/ab_$name.log 2>&1 || { tail -20 gpurun_out/ab_$name.log; return 1; }
  grep -E '^\[bench\] step|"metric"' gpurun_out/ab_$name.log | cut -c1-330
}
run sharedcached && run sharednt CFC_DECODE_SHARED_CACHED=0
