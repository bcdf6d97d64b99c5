# Round 3, GPU call c: the whole GPU suite, smoke, bench (default + forest walk-shape sweep,
# compact records), stream bench (default and from CDC wire columns).
set -eu
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --sweep-variant 1,3,4,5,6 > $O/bench_base.json 2> $O/bench_base.err
grep variant_sweep $O/bench_base.err || true
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --compact-records > $O/bench_compact.json 2> $O/bench_compact.err
for f in base compact; do python3 -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"; done
timeout -k 10 400 python3 bench_stream.py > $O/stream.json 2> $O/stream.err
cat $O/stream.json
timeout -k 10 400 python3 bench_stream.py --cdc > $O/stream_cdc.json 2> $O/stream_cdc.err
cat $O/stream_cdc.json
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 --sharded > $O/bench_sharded.json 2> $O/bench_sharded.err
python3 -c "import json; d=json.load(open('$O/bench_sharded.json')); print('sharded', d['ms_per_step'], json.dumps(d.get('exchange')))"
echo r03c done
