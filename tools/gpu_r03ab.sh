# Round 3, GPU call ab: row assembly segment counts by lane quads (16 lines per gather instead
# of 64) -- parity, A/B against per-lane gathers (FDX_ZFILL_QUAD=0).
set -eu
O=gpurun_out/r03ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_payload.py tests/test_gpu_distributed.py tests/test_gpu_edge.py tests/test_gpu_config1.py tests/test_gpu_scan.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" quad$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_zq0.so $B 2>/dev/null | python3 -c "$S" lane$r
done
echo r03ab done
