# Unrolled gathers in k_interleave and the k_terminal staging: parity, then bench breakdown.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r33.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r33.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r33.log
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r33.json 2> gpurun_out/bench_r33.err || exit 1
cat gpurun_out/bench_r33.json; grep breakdown gpurun_out/bench_r33.err
