# A/B: k_zfill_grouped_w3 on one resident round of blocks vs the stream grid (2,048 blocks).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r34.json 2> gpurun_out/bench_r34.err || exit 1
grep breakdown gpurun_out/bench_r34.err
FDX_PREP_FULL_GRID=1 timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r34g.json 2> gpurun_out/bench_r34g.err || exit 1
grep breakdown gpurun_out/bench_r34g.err
timeout -k 10 300 python -u bench.py --breakdown --no-cpu-baseline > gpurun_out/bench_r34b.json 2> gpurun_out/bench_r34b.err || exit 1
grep breakdown gpurun_out/bench_r34b.err
