"""Per-kernel summary of a rocprofv3 --kernel-trace CSV: all dispatches, and the dispatches
with the kernel's largest grid (the bench-size ones -- bench.py also runs the forest once on
its 4,096-row sklearn check sample, which the --stats average mixes in).

usage: python tools/trace_summary.py gpurun_out/prof_rNN [out.csv]
"""
import collections
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/*/*kernel_trace.csv")[0]
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(list)
    for r in rows:
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        per[r["Kernel_Name"]].append((g, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = []
    for name, v in per.items():
        gmax = max(g for g, _ in v)
        big = [d for g, d in v if g == gmax]
        out.append((sum(d for _, d in v), name, len(v), sum(d for _, d in v) / len(v) / 1e3, len(big),
                    sum(big) / len(big) / 1e3, gmax))
    out.sort(reverse=True)
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["kernel", "calls", "avg_us_all", "calls_max_grid", "avg_us_max_grid", "max_grid", "total_us"])
    for tot, name, n, avg, nb, avgb, g in out:
        w.writerow([name[:160], n, round(avg, 2), nb, round(avgb, 2), g, round(tot / 1e3, 1)])


if __name__ == "__main__":
    main()
