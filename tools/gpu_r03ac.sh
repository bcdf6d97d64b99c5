# Round 3, GPU call ac: 24-byte vs compact 16-byte terminal count records end to end.
set -eu
O=gpurun_out/r03ac
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2 3; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" rec24_$r
timeout -k 10 300 python3 $B --compact-records 2>/dev/null | python3 -c "$S" rec16_$r
done
echo r03ac done
