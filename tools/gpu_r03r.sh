# Round 3, GPU call r: PMC of HEAD (HBM bytes + SQ/LDS passes) and a kernel trace + timeline.
set -eu
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_base.json 2> $O/bench_base.err
python3 -c "import json; d=json.load(open('$O/bench_base.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt || true
bash tools/gpu_pmc.sh r03r sq
echo r03r done
