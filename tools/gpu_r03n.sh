# Round 3, GPU call l: critical chain on a pipeline-owned high-priority stream -- GPU suite, bench, timeline.
# customer rows are re-keyed -- GPU suite, bench, one step's timeline.
O=gpurun_out/r03n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_base.json 2> $O/bench_base.err
python3 -c "import json; d=json.load(open('$O/bench_base.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
head -62 $O/timeline.txt
echo r03n done
