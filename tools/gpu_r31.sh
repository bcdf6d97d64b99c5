# A/B of the pipelined W=3 prepare kernel (k_zfill_grouped_w3) vs the generic one; parity first.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r31.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r31.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r31.log
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r31.json 2> gpurun_out/bench_r31.err || exit 1
cat gpurun_out/bench_r31.json; grep breakdown gpurun_out/bench_r31.err
FDX_PREP_GENERIC=1 timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r31g.json 2> gpurun_out/bench_r31g.err || exit 1
grep breakdown gpurun_out/bench_r31g.err
timeout -k 10 400 python -u bench_stream.py > gpurun_out/stream_r31.log 2>&1 || exit 1
tail -1 gpurun_out/stream_r31.log
