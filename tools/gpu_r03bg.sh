# Round 3, GPU call bg: walk exit test every 4 (default) / 8 / 20 steps
# -- bench A/B only.
set -eu
O=gpurun_out/r03bg
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for v in default exit8 exit20; do
  if [ $v = default ]; then C="bench.py"; else C="tools/with_lib.py tools/ab/libfdx_$v.so bench.py"; fi
  timeout -k 10 300 python3 $C --steps 10 --warmup 3 --no-cpu-baseline --isolated-steps 1 > $O/bench_$v.json 2> $O/bench_$v.err || { echo bench failed; tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['traverse_ms'])" | tee -a $O/ab.txt
done
done
echo r03bg done
