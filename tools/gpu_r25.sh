timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r25.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r25.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r25.log
for c in 5000 20000; do
timeout -k 10 300 python -u bench.py --customers $c --terminals $((c*2)) --steps 3 --warmup 1 --no-cpu-baseline --sweep-variant 34,27 > gpurun_out/small_$c.json 2> gpurun_out/small_$c.err || exit 1
grep -o '"tx_per_gpu": [0-9]*' gpurun_out/small_$c.json; tail -1 gpurun_out/small_$c.err
done
