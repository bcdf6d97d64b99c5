timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_dist_r21.log 2>&1 || { tail -30 gpurun_out/pytest_dist_r21.log; exit 1; }
tail -2 gpurun_out/pytest_dist_r21.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --sharded > gpurun_out/sharded_r21.json 2> gpurun_out/sharded_r21.err || exit 1
cat gpurun_out/sharded_r21.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r21 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sharded > gpurun_out/prof_r21.log 2>&1
