"""Timeline of one bench.py step from a rocprofv3 --kernel-trace (csv): every dispatch of the
step with its start / end relative to the step start (µs), its hardware queue, and the idle
gaps between dispatches.  Steps are delimited by the forest's launches: the step is the
dispatches after the (k-1)-th run of k_forest_rank launches up to the end of the k-th.

usage: python tools/step_timeline.py gpurun_out/<dir> [step_index (default 2)]
"""
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ends = []  # index of the last k_forest_rank of each run of consecutive forest launches
    for i, r in enumerate(rows):
        if "k_forest_rank" in r["Kernel_Name"] and (i + 1 == len(rows) or "k_forest_rank" not in rows[i + 1]["Kernel_Name"]):
            ends.append(i)
    lo, hi = ends[k - 1] + 1, ends[k]
    step = rows[lo:hi + 1]
    t0 = int(step[0]["Start_Timestamp"])
    qkey = "Queue_Id" if "Queue_Id" in step[0] else ("Stream_Id" if "Stream_Id" in step[0] else None)
    busy_end = t0
    print(f"{'start':>9} {'end':>9} {'dur':>8} {'gap':>7}  queue  kernel")
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - busy_end)
        busy_end = max(busy_end, e)
        name = r["Kernel_Name"].replace("fdx::(anonymous namespace)::", "").split("(")[0]
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap / 1e3:7.1f}  {r.get(qkey, '-') if qkey else '-':>5}  {name[:70]}")
    print(f"step: {(busy_end - t0) / 1e3:.1f} µs over {len(step)} dispatches")


if __name__ == "__main__":
    main()
