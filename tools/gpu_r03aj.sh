# Round 3, GPU call aj: row assembly's segment loads nontemporal (study build).
set -eu
O=gpurun_out/r03aj
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if r['stage'] == 'assemble_rows'])"
B="bench.py --no-cpu-baseline --steps 5 --warmup 2"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" base$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_ntseg.so $B 2>/dev/null | python3 -c "$S" ntseg$r
done
echo r03aj done
