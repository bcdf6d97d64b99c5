# Round 3, GPU call ar: re-key probe + kernel trace of one bench step (customer re-key timing check).
set -eu
O=gpurun_out/r03ar
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do timeout -k 10 300 python3 tools/radix_ab.py 2>/dev/null; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r03ar/kt/*/*_kernel_stats.csv"):
    for r in csv.reader(open(f)):
        if any(k in r[0] for k in ("seg_", "radix", "scan_", "plan_small", "fillBuffer")):
            print(r[0].split("(")[0].replace("fdx::", "")[-45:], r[1], "avg_us", round(float(r[3]) / 1000, 1))
PY
echo r03ar done
