bash tools/gpu_round.sh r17 || exit 1
FDX_CUSTOMER_WALK=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/walk0.json 2> gpurun_out/walk0.err || exit 1
tail -1 gpurun_out/walk0.err
