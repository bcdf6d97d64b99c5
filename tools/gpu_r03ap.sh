# Round 3, GPU call ap: layout plan phases 3/4 trimmed -- plan order tests, probe, bench.
set -eu
O=gpurun_out/r03ap
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config1.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/probe -- python3 $GRAFT_REPO_ROOT/tools/plan_probe.py > $GRAFT_REPO_ROOT/$O/probe.log 2>&1
cd $GRAFT_REPO_ROOT
grep -h "k_layout_plan_small" $O/probe/*/*_kernel_stats.csv | cut -d, -f2-4
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if r['stage'] == 'customer_layout'])"
for r in 1 2 3; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "$S" b$r
done
echo r03ap done
