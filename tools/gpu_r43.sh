# k_prepare with wave-uniform integer rank tables: full GPU parity suite, then configs[2] forest bench (100M rows).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_r43.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r43.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r43.log
timeout -k 10 300 python -u bench_forest.py > gpurun_out/forest100m_r43.json 2> gpurun_out/forest100m_r43.err \
    || { tail -20 gpurun_out/forest100m_r43.err; exit 1; }
cat gpurun_out/forest100m_r43.json
