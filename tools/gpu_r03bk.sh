# Round 3, GPU call bk: rocprofv3 kernel trace + stats of the default bench on the final HEAD
# (the k_forest_rank average behind the bench line's roofline) and the step timeline.
set -eu
O=gpurun_out/r03bk
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ktrace -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/ktrace_bench.json 2> $GRAFT_REPO_ROOT/$O/ktrace.log
cd $GRAFT_REPO_ROOT
python3 tools/step_timeline.py $O/ktrace 2 > $O/timeline.txt
grep -i forest $(find $O/ktrace -name "*kernel_stats.csv") | head -3
python3 -c "import json; d=json.load(open('$O/ktrace_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
echo r03bk done
