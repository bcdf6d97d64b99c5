# A/B of the two-class terminal kernel (512-row LDS stage for short segments) vs one 1,024-row stage.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r32.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r32.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r32.log
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r32.json 2> gpurun_out/bench_r32.err || exit 1
cat gpurun_out/bench_r32.json; grep breakdown gpurun_out/bench_r32.err
FDX_TERM_ONE_STAGE=1 timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r32g.json 2> gpurun_out/bench_r32g.err || exit 1
grep breakdown gpurun_out/bench_r32g.err
