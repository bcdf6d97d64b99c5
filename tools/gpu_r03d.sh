# Round 3, GPU call d: variant table after the prune (default 10 chains), forest bench on the
# bench model and the deployed model per walk variant, kernel-trace stats of the bench, PMC
# passes (HBM bytes + SQ/LDS) on HEAD.
set -eu
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --sweep-variant 1,2,3,4,5,6,7,8,9 > $O/bench_base.json 2> $O/bench_base.err
grep variant_sweep $O/bench_base.err || true
python3 -c "import json; d=json.load(open('$O/bench_base.json')); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step']) for r in d['kernels']['per_stage']])"
for v in 1 2 8; do timeout -k 10 200 python3 bench_forest.py --rows 20000000 --variant $v > $O/forest_v$v.json 2>> $O/forest.err; done
for v in 2 8 3 9; do timeout -k 10 200 python3 bench_forest.py --rows 20000000 --model bench_assets/rf_deployed.npz --variant $v > $O/forest_dep_v$v.json 2>> $O/forest.err; done
for f in $O/forest_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['variant'], d['prepare_ms'], d['traverse_ms'])"; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/ktrace.log 2>&1
cd $GRAFT_REPO_ROOT
bash tools/gpu_pmc.sh r03d sq
echo r03d done
