for wk in 256 1; do
  FDX_CUSTOMER_WALK=$wk timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/walk$wk.json 2> gpurun_out/walk$wk.err || exit 1
  tail -1 gpurun_out/walk$wk.err
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FDX_CUSTOMER_WALK=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r18 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r18.log 2>&1
