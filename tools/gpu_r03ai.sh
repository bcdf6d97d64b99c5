# Round 3, GPU call ai: where the row assembly's time goes -- study builds (wrong outputs,
# timing only): no Eytzinger descent (noeytz), no segment loads (noseg), neither (nosearch).
set -eu
O=gpurun_out/r03ai
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if r['stage'] == 'assemble_rows'])"
B="bench.py --no-cpu-baseline --steps 5 --warmup 2"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" base$r
for v in noeytz noseg nosearch; do
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_$v.so $B 2>/dev/null | python3 -c "$S" $v$r
done
done
echo r03ai done
