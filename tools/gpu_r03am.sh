# Round 3, GPU call am: radix histogram by LDS atomics vs ballot multisplit.
set -eu
O=gpurun_out/r03am
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python3 tools/radix_ab.py --out /tmp/p_base.pt 2>/dev/null | sed "s/^/base /"
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_hatom.so tools/radix_ab.py --out /tmp/p_hatom.pt 2>/dev/null | sed "s/^/hatom /"
done
python3 tools/radix_ab.py --compare /tmp/p_base.pt /tmp/p_hatom.pt
S="import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['ms_per_step'], [(r['stage'], r.get('ms_isolated')) for r in d['kernels']['per_stage'] if 'rekey' in r['stage']])"
for r in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "$S" base$r
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_hatom.so bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "$S" hatom$r
done
echo r03am done
