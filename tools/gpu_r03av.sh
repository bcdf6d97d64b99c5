# Round 3, GPU call av: lane-paced walk with an advance threshold (variants 11-18) -- parity tests, variant sweep, bench with variant 11.
set -eu
O=gpurun_out/r03av
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_forest_lanes.py "tests/test_gpu_parity.py::test_fused_scoring_every_rank_format" -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --sweep-variant 1,11,16,17,18,12 > $O/sweep.json 2> $O/sweep.err || { echo sweep failed; tail -20 $O/sweep.err; exit 1; }
grep -i "variant" $O/sweep.err | tail -12 || true
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --forest-variant 11 > $O/bench11.json 2> $O/bench11.err || { echo bench failed; tail -20 $O/bench11.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench11.json')); print('v11', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['traverse_ms'])"
echo r03av done
