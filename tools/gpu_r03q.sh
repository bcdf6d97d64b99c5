# Round 3, GPU call q: XCD-aware radix scatter tiles (A/B build), bit-equality + timing.
set -eu
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python3 tools/radix_ab.py --out $O/base.pt 2>/dev/null | tee $O/radix_base$r.json
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_xcd.so tools/radix_ab.py --out $O/xcd.pt 2>/dev/null | tee $O/radix_xcd$r.json
done
python3 tools/radix_ab.py --compare $O/base.pt $O/xcd.pt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('base', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
timeout -k 10 300 python3 tools/with_lib.py tools/ab/libfdx_xcd.so bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xcd', d['ms_per_step'], [(r['stage'], r['ms_in_step'], r.get('ms_isolated')) for r in d['kernels']['per_stage']])"
echo r03q done
