bash tools/gpu_round.sh r16 || exit 1
for rg in 64 128; do
  FDX_CUSTOMER_RING=$rg timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/ring_$rg.json 2> gpurun_out/ring_$rg.err || exit 1
  tail -1 gpurun_out/ring_$rg.err
done
