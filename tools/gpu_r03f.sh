# Round 3, GPU call f: register-rank forest walk (variants 10-12) -- parity, then the sweep.
set -eu
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --sweep-variant 1,5,10,11,12 > $O/bench_base.json 2> $O/bench_base.err
grep variant_sweep $O/bench_base.err || true
for v in 1 10 11; do timeout -k 10 200 python3 bench_forest.py --rows 20000000 --variant $v > $O/forest_v$v.json 2>> $O/forest.err; python3 -c "import json; d=json.load(open('$O/forest_v$v.json')); print('forest', d['variant'], d['prepare_ms'], d['traverse_ms'])"; done
echo r03f done
