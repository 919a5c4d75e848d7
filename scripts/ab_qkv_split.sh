set -o pipefail
mkdir -p gpurun_out
for s in 0 2 8 0 2 8; do
  CFC_DECODE_QKV_SPLIT=$s timeout -k 10 300 python bench.py --llm-only --steps 2 --warmup 1 --latency-rate 0 --latency-low-rate 0 --service-latency-rate 0 > gpurun_out/ab_qkv_$s.out 2> gpurun_out/ab_qkv_$s.err || exit $?
  echo "split=$s $(grep -o 'decode=[0-9.]*s' gpurun_out/ab_qkv_$s.err | tr '\n' ' ')" | tee -a gpurun_out/r05_ab_qkv_split.log
done
