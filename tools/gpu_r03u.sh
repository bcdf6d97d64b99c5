# Round 3, GPU call u: id range checks folded into the re-keys -- parity tests, bench, timeline.
set -eu
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_payload.py tests/test_gpu_distributed.py tests/test_gpu_edge.py tests/test_gpu_config1.py tests/test_gpu_dropin.py tests/test_gpu_configs.py::test_fused_path_rejects_ids_out_of_range -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_base.json 2> $O/bench_base.err
python3 -c "import json; d=json.load(open('$O/bench_base.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"

cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
awk '$3>15' $O/timeline.txt | head -24

timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 --sharded > $O/bench_sharded.json 2> $O/bench_sharded.err
python3 -c "import json; d=json.load(open('$O/bench_sharded.json')); print('sharded', d['ms_per_step'], d['exchange']['per_rank'][0]['hidden_share'])"
echo r03u done
