# Re-key parity incl. the new 9-bit-digit cases (18- and 25-bit keys).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "rekey" > gpurun_out/pytest_r40.log 2>&1 || { tail -30 gpurun_out/pytest_r40.log; exit 1; }
grep -c PASSED gpurun_out/pytest_r40.log; tail -1 gpurun_out/pytest_r40.log
