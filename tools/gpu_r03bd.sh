# Round 3, GPU call bd: the first tile fetched before the node fill -- forest parity tests, bench, kernel trace.
set -eu
O=gpurun_out/r03bd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_forest_onegroup.py tests/test_gpu_parity.py tests/test_gpu_config1.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --sweep-variant 1,4 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
grep -i "variant_sweep" $O/bench.err | tail -3 || true
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['traverse_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace_bench.json 2> $GRAFT_REPO_ROOT/$O/ktrace.log
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
grep forest $O/timeline.txt | head -20
echo r03bd done
