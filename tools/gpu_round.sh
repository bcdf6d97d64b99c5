# One GPU session: parity tests, bench (+ variant sweep), rocprof kernel summary.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
mkdir -p gpurun_out
TAG=${1:-rx}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --breakdown --sweep-variant ${VARIANTS:-1} > gpurun_out/bench_$TAG.json \
    2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof exit $?"
python tools/trace_summary.py gpurun_out/prof_$TAG gpurun_out/prof_$TAG/trace_summary.csv || true
