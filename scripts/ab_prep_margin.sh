# A/B of the just-in-time preparation lead (bench_pipeline.py CFC_PREP_MARGIN / CFC_PREP_SLACK_S):
# 20 timed steps + 5 warm-up each, throughput half only; reports value, p50 and the summed wait_prep.
set -o pipefail
mkdir -p gpurun_out
for cfg in "2.0 0.25" "1.25 0.1" "2.0 0.25" "1.25 0.1"; do
  set -- $cfg
  CFC_PREP_MARGIN=$1 CFC_PREP_SLACK_S=$2 timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 \
    --latency-rate 0 --service-latency-rate 0 > gpurun_out/ab_prep.out 2> gpurun_out/ab_prep.err || exit 1
  python - "$1" "$2" >> gpurun_out/r05_ab_prep_margin.log <<'PY'
import json, re, sys
d = json.loads(open("gpurun_out/ab_prep.out").read().strip().splitlines()[-1])
w = sum(float(x) for x in re.findall(r"wait_prep=([0-9.]+)s", open("gpurun_out/ab_prep.err").read()))
print(f"margin={sys.argv[1]} slack={sys.argv[2]} value={d['value']} p50={d['p50_summary_latency_s']} "
      f"ms_per_step={d['ms_per_step']} wait_prep_sum={w:.2f}s", flush=True)
PY
done
cat gpurun_out/r05_ab_prep_margin.log
