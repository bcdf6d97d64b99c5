# Round 3, GPU call e: fair forest-variant sweep (two rounds, warm), kernel-trace stats of the
# bench, PMC passes (HBM bytes + SQ/LDS) on HEAD.
set -eu
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --sweep-variant 1,4,5,6,7,3,9 > $O/bench_base.json 2> $O/bench_base.err
grep variant_sweep $O/bench_base.err || true
python3 -c "import json; d=json.load(open('$O/bench_base.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step']) for r in d['kernels']['per_stage']])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
bash tools/gpu_pmc.sh r03e sq
echo r03e done
