timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k variants --timeout 120 --timeout-method thread > gpurun_out/pytest_var_r26.log 2>&1 || { tail -30 gpurun_out/pytest_var_r26.log; exit 1; }
tail -1 gpurun_out/pytest_var_r26.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --sweep-variant 34,41,42,43,34 > gpurun_out/sw_r26.json 2> gpurun_out/sw_r26.err || exit 1
tail -1 gpurun_out/sw_r26.err
