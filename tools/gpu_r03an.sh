# Round 3, GPU call an: k_seg_mark4 (4 keys per thread) -- parity, bench, timeline.
set -eu
O=gpurun_out/r03an
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_payload.py tests/test_gpu_edge.py tests/test_gpu_config1.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if 'rekey' in r['stage']])"
for r in 1 2 3; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "$S" b$r
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
grep -E "seg_|plan|interleave|terminal_short|zfill" $O/timeline.txt
echo r03an done
