VARIANTS=23,27,31,32,33,34,35 bash tools/gpu_round.sh r15 || exit 1
for sp in 0 100000 500; do
  FDX_CUSTOMER_RING_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/split_$sp.json 2> gpurun_out/split_$sp.err || exit 1
  tail -1 gpurun_out/split_$sp.err
done
