# Round 3, GPU call x: the terminal records' scatter with 8-byte records (study build).
set -eu
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" base$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_rec8.so $B 2>/dev/null | python3 -c "$S" rec8_$r
done
echo r03x done
