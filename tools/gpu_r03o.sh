# Round 3, GPU call o: mixed register / plane chains in the forest walk (variants 11-13).
set -eu
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --sweep-variant 1,11,12,13,5 > $O/bench_base.json 2> $O/bench_base.err
grep variant_sweep $O/bench_base.err || true
echo r03o done
