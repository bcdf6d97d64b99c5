# Round 3, GPU call bb: PMC of HEAD (one-group forest tile loop) (FETCH/WRITE + SQ passes), kernel-trace stats and the step
# timeline of the default bench.
set -eu
O=gpurun_out/r03bb
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_pmc.sh r03bb sq
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/ktrace_bench.json 2> $GRAFT_REPO_ROOT/$O/ktrace.log
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
awk '$3>15' $O/timeline.txt > $O/timeline_top.txt
head -30 $O/timeline_top.txt
echo r03bb done
