#!/bin/bash
# rocprofv3 kernel-trace + stats of a short LLM bench (decode-heavy and prefill phases).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
rm -rf gpurun_out/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py "$@" > gpurun_out/prof_bench.log 2>&1; rc=$?
tail -3 gpurun_out/prof_bench.log
[ $rc -eq 0 ] || exit $rc
python scripts/prof_summary.py gpurun_out/prof gpurun_out/prof_summary.txt > /dev/null
cat gpurun_out/prof_summary.txt | head -40
# the raw per-dispatch trace is hundreds of MB: keep only the stats so gpurun_out/ is copied back
find gpurun_out/prof -name '*kernel_trace.csv' -delete
