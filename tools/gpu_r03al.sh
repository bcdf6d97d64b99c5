# Round 3, GPU call al: range-check copy behind the layout plan.
set -eu
O=gpurun_out/r03al
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "layout or fused" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'])"
for r in 1 2 3; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "$S" poll$r
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
awk '$1>900 && $1<1400' $O/timeline.txt
echo r03al done
