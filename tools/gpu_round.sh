# One GPU session: parity tests, bench (+ variant sweep), rocprof kernel summary.
set -u
mkdir -p gpurun_out
TAG=${1:-rx}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_$TAG.log
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 600 python bench.py --breakdown --sweep-variant ${VARIANTS:-0,1,2,3,4} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof exit $?"
