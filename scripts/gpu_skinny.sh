set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "skinny or silu" > gpurun_out/pytest_skinny.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_skinny.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_skinny.py 1 8 64 128 256 > gpurun_out/bench_skinny.log 2>&1; rc=$?; cat gpurun_out/bench_skinny.log | tail -30; exit $rc
