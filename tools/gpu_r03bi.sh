# Round 3, GPU call bi: adaptive unchecked walk prefix in whole unrolled intervals (the previous tile's steps less one exit
# interval) -- forest / parity / config-1 GPU tests, bench x2.
set -eu
O=gpurun_out/r03bi
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_forest_onegroup.py tests/test_gpu_parity.py tests/test_gpu_config1.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --isolated-steps 1 > $O/bench_$i.json 2> $O/bench_$i.err || { echo bench failed; tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print('adaptive', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['traverse_ms'])" | tee -a $O/ab.txt
done
echo r03bi done
