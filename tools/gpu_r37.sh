# Experiment: k_interleave with both gathers on one line per row (amount read from ts: wrong
# values, timing only) vs normal.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline --steps 5 > gpurun_out/bench_r37.json 2> gpurun_out/bench_r37.err || exit 1
grep breakdown gpurun_out/bench_r37.err
FDX_EXP_ONE_LINE=1 timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline --steps 5 > gpurun_out/bench_r37x.json 2> gpurun_out/bench_r37x.err || exit 1
grep breakdown gpurun_out/bench_r37x.err
