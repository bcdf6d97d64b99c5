# Re-verify HEAD on a fresh box: smoke, parity tests, bench + rocprof, config-5 stream bench, PMC passes.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r39.log 2>&1 || exit 1
bash tools/gpu_round.sh r39 || exit 1
timeout -k 10 400 python -u bench_stream.py > gpurun_out/stream_r39.log 2>&1 || exit 1
bash tools/gpu_pmc.sh r39
