# Round 3, GPU call af: row assembly held to 128 VGPRs (4 waves per SIMD, FDX_ZFILL_WAVES=4) vs
# the compiler's 156 (3 waves).
set -eu
O=gpurun_out/r03af
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if r['stage'] == 'assemble_rows'])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2 3; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" base$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_zw4.so $B 2>/dev/null | python3 -c "$S" w4_$r
done
echo r03af done
