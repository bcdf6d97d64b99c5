# Final check of HEAD's build: smoke, full GPU suite, default bench.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r44.log 2>&1 || { tail -20 gpurun_out/smoke_r44.log; exit 1; }
tail -1 gpurun_out/smoke_r44.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r44.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r44.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r44.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r44.json 2> gpurun_out/bench_r44.err || exit 1
cat gpurun_out/bench_r44.json
