# Round 3, GPU call be: forest rows in MALL-sized parts (each part walks every chunk before the
# next) -- forest parity tests, then bench A/B: 4M-row parts (default) / no split / 2M-row parts.
set -eu
O=gpurun_out/r03be
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_forest_onegroup.py tests/test_gpu_parity.py tests/test_gpu_config1.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for v in default nosplit part2m; do
  if [ $v = default ]; then C="bench.py"; else C="tools/with_lib.py tools/ab/libfdx_$v.so bench.py"; fi
  timeout -k 10 300 python3 $C --steps 10 --warmup 3 --no-cpu-baseline --isolated-steps 1 > $O/bench_$v.json 2> $O/bench_$v.err || { echo bench failed; tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['traverse_ms'])" | tee -a $O/ab.txt
done
done
echo r03be done
