# New overflow parity test, then the full GPU suite and the default bench (with the LDS roofline).
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "overflows" > gpurun_out/pytest_r36_new.log 2>&1 || { tail -40 gpurun_out/pytest_r36_new.log; exit 1; }
tail -2 gpurun_out/pytest_r36_new.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r36.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r36.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r36.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r36.json 2> gpurun_out/bench_r36.err || exit 1
cat gpurun_out/bench_r36.json
