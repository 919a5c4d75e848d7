set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_custom_ar_gpu.py -x -v --timeout 700 --timeout-method thread > gpurun_out/r05_tp_overlap_tests.log 2>&1 || { tail -30 gpurun_out/r05_tp_overlap_tests.log; exit 1; }
tail -3 gpurun_out/r05_tp_overlap_tests.log
CFC_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --tp 2 --steps 2 --warmup 1 --latency-rate 0 --service-latency-rate 0 > gpurun_out/r05_bench_tp2_overlap.out 2> gpurun_out/r05_bench_tp2_overlap.err
