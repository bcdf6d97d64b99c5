# Round 3, GPU call m: caller-stream priority A/B (the customer half is the critical path).
set -eu
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config1.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_base$r.json 2> $O/bench_base$r.err
python3 -c "import json; d=json.load(open('$O/bench_base$r.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step']) for r in d['kernels']['per_stage']])"
timeout -k 10 300 python3 tools/prio_ab.py -1 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_hi$r.json 2> $O/bench_hi$r.err
python3 -c "import json; d=json.load(open('$O/bench_hi$r.json')); print('main_high', d['ms_per_step'], [(r['stage'], r['ms_in_step']) for r in d['kernels']['per_stage']])"
done
echo r03m done
