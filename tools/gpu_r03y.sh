# Round 3, GPU call y: radix scatter payload prefetch A/B (0: after each phase, 1: default, 2: with the keys).
set -eu
O=gpurun_out/r03y
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python3 tools/radix_ab.py --out /tmp/p1.pt 2>/dev/null | sed "s/^/p1 /"
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_rp0.so tools/radix_ab.py --out /tmp/p0.pt 2>/dev/null | sed "s/^/p0 /"
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_rp2.so tools/radix_ab.py --out /tmp/p2.pt 2>/dev/null | sed "s/^/p2 /"
done
python3 tools/radix_ab.py --compare /tmp/p0.pt /tmp/p1.pt
python3 tools/radix_ab.py --compare /tmp/p0.pt /tmp/p2.pt
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
B="bench.py --no-cpu-baseline --steps 10 --warmup 3"
for r in 1 2; do
timeout -k 10 300 python3 $B 2>/dev/null | python3 -c "$S" p1_$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_rp0.so $B 2>/dev/null | python3 -c "$S" p0_$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_rp2.so $B 2>/dev/null | python3 -c "$S" p2_$r
done
echo r03y done
