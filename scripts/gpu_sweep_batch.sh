#!/bin/bash
# throughput / p50-latency operating curve of the headline pipeline vs threads per GPU
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for b in 64 128 192 256; do
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 --threads-per-gpu $b > gpurun_out/sweep_b$b.log 2>&1 || exit 1
  python - "$b" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/sweep_b{sys.argv[1]}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"B={sys.argv[1]:>4} threads/s={d['value']:.2f} p50={d['p50_summary_latency_s']:.2f}s ms/step={d['ms_per_step']}")
PY
done
