# Round 3, GPU call bl: stream priorities with the terminal half critical (final library):
# (crit, side) = (-1, 0) default / (-1, -1) equal / (0, -1) flipped, two rounds.
set -eu
O=gpurun_out/r03bl
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
for pr in "-1 0" "-1 -1" "0 -1"; do
  tag=$(echo $pr | tr ' ' '_')
  timeout -k 10 300 python3 tools/stream_prio_flip.py $pr bench.py --steps 10 --warmup 3 --no-cpu-baseline --isolated-steps 1 > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo bench failed; tail -20 $O/bench_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); print('prio $pr', d['ms_per_step'])" | tee -a $O/ab.txt
done
done
echo r03bl done
