# Round 3, GPU call g: LDS-only start / window searches (no flat loads) -- full GPU suite, bench.
set -eu
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_base.json 2> $O/bench_base.err
python3 -c "import json; d=json.load(open('$O/bench_base.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
echo r03g done
