#!/bin/bash
# IVF on MiniLM-tiled data with copy noise well below the spread of the distinct encodings (0.003
# per dimension, ~0.06 in norm), 300k distinct chunks; then the repeated dgemm X-first probe.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/bench_ivf.py --n 1e7 --data minilm --unique 300000 --noise 0.003 --out gpurun_out/ivf_r04d.jsonl > gpurun_out/ivf_minilm_d.log 2>&1 || { tail -20 gpurun_out/ivf_minilm_d.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/ivf_r04d.jsonl'):
    d=json.loads(l); print(d['data'], d['nprobe'], d['recall_at_10'], d['ms_per_16q'], d['flat_ms_per_16q'], d['rows_scanned_per_16q'], d['largest_list'], d['empty_lists'], d['encoder_s'])
"
bash scripts/gpu_r04_xfirst.sh
