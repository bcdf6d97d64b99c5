# Round 3, GPU call aq: segment offsets in one pass (no search) + layout plan trims -- parity,
# plan probe, bench, timeline.
set -eu
O=gpurun_out/r03aq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_payload.py tests/test_gpu_edge.py tests/test_gpu_config1.py tests/test_gpu_distributed.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/probe -- python3 $GRAFT_REPO_ROOT/tools/plan_probe.py > $GRAFT_REPO_ROOT/$O/probe.log 2>&1
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r03aq/probe/*/*_kernel_stats.csv"):
    for r in csv.reader(open(f)):
        if "plan_small" in r[0] or "seg_bounds" in r[0]:
            print(r[0].split("(")[0][-40:], r[1], "avg_us", round(float(r[3]) / 1000, 1))
PY
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if r['stage'] in ('rekey_customer','customer_layout','rekey_terminal')])"
for r in 1 2 3; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "$S" b$r
done
echo r03aq done
