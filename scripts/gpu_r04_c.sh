#!/bin/bash
# Round-4 (c): pgemm / IVF GPU tests with the W1-early default, centered-IVF on MiniLM-tiled 10M,
# headline bench (3 steps) with the current defaults.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -q -x --timeout 200 --timeout-method thread -k "pgemm or ivf or prefill or decode" > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -1 gpurun_out/c_tests.log
timeout -k 10 600 python -u scripts/bench_ivf.py --n 1e7 --data minilm --unique 100000 --out gpurun_out/ivf_r04c.jsonl > gpurun_out/ivf_minilm_c.log 2>&1 || { tail -20 gpurun_out/ivf_minilm_c.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/ivf_r04c.jsonl'):
    d=json.loads(l); print(d['data'], d['nprobe'], d['recall_at_10'], d['ms_per_16q'], d['flat_ms_per_16q'], d['rows_scanned_per_16q'], d['largest_list'], d['empty_lists'])
"
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_r04c.log 2>&1 || { tail -20 gpurun_out/bench_r04c.log; exit 1; }
grep -E '^\[bench\] step|"metric"' gpurun_out/bench_r04c.log | cut -c1-400
