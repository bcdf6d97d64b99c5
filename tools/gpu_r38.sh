# 9-bit radix digits for 17-18-bit keys (terminal re-key in 2 passes): parity, then A/B bench.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r38.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r38.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r38.log
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r38.json 2> gpurun_out/bench_r38.err || exit 1
grep breakdown gpurun_out/bench_r38.err; cut -c1-200 gpurun_out/bench_r38.json
FDX_RADIX_8BIT=1 timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r38g.json 2> gpurun_out/bench_r38g.err || exit 1
grep breakdown gpurun_out/bench_r38g.err
