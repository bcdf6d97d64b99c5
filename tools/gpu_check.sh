# One GPU round-trip: GPU tests, smoke, the default bench line, a rocprofv3 kernel trace of
# the bench.  Every GPU step has its own time limit; the first failure ends the script.
# usage (through gpurun): bash tools/gpu_check.sh <tag> [pytest selection]
set -eu
TAG=${1:?tag}
SEL=${2:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
cat gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_trace.log 2>&1
echo done
