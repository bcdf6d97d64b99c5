# Round 3, GPU call aa: scoring rows as two halves (customer half while the terminal windows run,
# terminal half after) -- parity, A/B against one assembly kernel, timeline.
set -eu
O=gpurun_out/r03aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_payload.py tests/test_gpu_distributed.py tests/test_gpu_edge.py tests/test_gpu_config1.py tests/test_gpu_dropin.py tests/test_gpu_scan.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" split$r
timeout -k 10 300 python3 tools/split_rows_ab.py 0 $B 2>/dev/null | python3 -c "$S" one$r
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
awk '$3>15' $O/timeline.txt > $O/timeline_top.txt
head -30 $O/timeline_top.txt
echo r03aa done
