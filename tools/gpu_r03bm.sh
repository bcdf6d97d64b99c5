# Round 3, GPU call bm: configs[2] forest bench (RF(100, d20) predict_proba over 100M resident rows) on the final library.
set -eu
O=gpurun_out/r03bm
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench_forest.py > $O/forest100m.json 2> $O/forest100m.err || { echo bench_forest failed; tail -20 $O/forest100m.err; exit 1; }
cat $O/forest100m.json | head -c 800; echo
echo r03bm done
