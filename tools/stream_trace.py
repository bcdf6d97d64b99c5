"""Per-kernel times of the timed micro-batches in a rocprofv3 --kernel-trace of
bench_stream.py: dispatches after the last history-sized k_stream_process (the history is
streamed in day-sized batches first), grouped by kernel, with the per-batch sum.

usage: python tools/stream_trace.py gpurun_out/prof_stream [out.csv] [n_batches]
(n_batches: the timed + warm-up micro-batches at the end of the trace, default 30)
"""
import collections
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/*/*kernel_trace.csv")[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    link = [i for i, r in enumerate(rows) if "k_stream_link" in r["Kernel_Name"]]
    tail = rows[link[-nb]:]
    n_batches = sum(1 for r in tail if "k_stream_process" in r["Kernel_Name"])
    per = collections.defaultdict(list)
    for r in tail:
        per[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["kernel", "calls", "avg_us", "us_per_batch"])
    tot = 0.0
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        pb = sum(v) / 1e3 / max(n_batches, 1)
        tot += pb
        w.writerow([name[:120], len(v), round(sum(v) / len(v) / 1e3, 2), round(pb, 2)])
    w.writerow(["(all kernels)", "", "", round(tot, 2)])
    w.writerow(["(micro-batches)", n_batches, "", ""])


if __name__ == "__main__":
    main()
