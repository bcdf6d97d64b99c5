"""rocprofv3 CSVs of tools/fetch_calib (FETCH_SIZE pass, WRITE_SIZE pass, kernel trace) ->
profiles/<tag>_fetch_calibration.json: per access shape, the raw counter, the known or
minimum byte count, their ratio, and the kernel's duration and implied byte rate.

usage: python tools/fetch_calib_report.py gpurun_out/<tag>_calib out.json
(reads <prefix>_fetch, <prefix>_write, <prefix>_trace)"""
import collections
import csv
import glob
import json
import sys

GIB = 2 << 30
M = 64 << 20
KNOWN = {  # kernel -> (known bytes read, known bytes written, what)
    "stream16": (GIB, 0, "coalesced 16 B/lane reads"),
    "stream8": (GIB, 0, "coalesced 8 B/lane reads"),
    "stream4": (GIB, 0, "coalesced 4 B/lane reads"),
    "gather<1>": (M * 8, 0, "random 8 B reads (useful bytes; >= 1 line each)"),
    "gather<2>": (M * 16, 0, "random 16 B reads"),
    "gather<3>": (M * 24, 0, "random 24 B record reads"),
    "scatter24": (0, M * 24, "random 24 B record writes"),
    "write16": (0, GIB, "coalesced 16 B/lane writes"),
}


def second_dispatch(prefix, counter=None):
    f = glob.glob(prefix + "/*/*counter_collection.csv") if counter else glob.glob(prefix + "/*/*kernel_trace.csv")
    rows = list(csv.DictReader(open(f[0])))
    seen = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].removeprefix("void ")
        key = next((k for k in KNOWN if name.startswith(k.split("<")[0]) and (("<" not in k) or k in name)), None)
        if key is None:
            continue
        if counter:
            if r["Counter_Name"] == counter:
                seen[key].append(float(r["Counter_Value"]))
        else:
            seen[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: v[-1] for k, v in seen.items()}


def main():
    pre, out = sys.argv[1], sys.argv[2]
    fetch = second_dispatch(pre + "_fetch", "FETCH_SIZE")
    write = second_dispatch(pre + "_write", "WRITE_SIZE")
    dur = second_dispatch(pre + "_trace")
    res = {}
    for k, (rd, wr, what) in KNOWN.items():
        e = {"what": what, "duration_s": dur.get(k)}
        if k in fetch:
            e["FETCH_SIZE_bytes"] = fetch[k] * 1024
            if rd:
                e["fetch_over_known"] = round(fetch[k] * 1024 / rd, 4)
        if k in write:
            e["WRITE_SIZE_bytes"] = write[k] * 1024
            if wr:
                e["write_over_known"] = round(write[k] * 1024 / wr, 4)
        if dur.get(k):
            e["known_GBs"] = round((rd + wr) / dur[k] / 1e9, 1)
            if k.startswith("gather") or k == "scatter24":
                e["accesses_per_s"] = round(M / dur[k] / 1e9, 3)
        res[k] = e
    with open(out, "w") as f:
        json.dump({"source": "tools/fetch_calib.hip under rocprofv3 (separate FETCH_SIZE / WRITE_SIZE passes + "
                             "kernel trace), 1x MI355X, second of two repetitions", "kernels": res}, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
