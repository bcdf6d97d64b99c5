# Round 3, GPU call w: stream-priority A/B with the terminal half critical; the cost of the
# terminal records' random scatter (sequential-store study build).
set -eu
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" base$r
timeout -k 10 300 python3 tools/stream_prio_ab.py -1 -1 $B 2>/dev/null | python3 -c "$S" both_hi$r
timeout -k 10 300 python3 tools/stream_prio_ab.py 0 -1 $B 2>/dev/null | python3 -c "$S" side_hi$r
timeout -k 10 300 python3 tools/stream_prio_ab.py 0 0 $B 2>/dev/null | python3 -c "$S" both_lo$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_tsseq.so $B 2>/dev/null | python3 -c "$S" seqstore$r
done
echo r03w done
