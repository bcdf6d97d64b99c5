set -u
mkdir -p gpurun_out
for R in 192 96 48; do
  FDX_CUSTOMER_RING=$R timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --breakdown > gpurun_out/ring_$R.json 2> gpurun_out/ring_$R.err || exit 1
  grep breakdown gpurun_out/ring_$R.err
done
