"""Summarise rocprofv3 --pmc CSVs per kernel (per-dispatch means over the bench-size
dispatches, i.e. those with the kernel's largest grid), and derive HBM traffic the way
MI355X_MICROARCH.md prescribes: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reads half the bytes of wide coalesced streaming reads, so traffic = 2*FETCH + WRITE
(upper estimate for the read side; ratios between variants are unaffected).

usage: python tools/pmc_summary.py gpurun_out/pmc_r7 [kernel-substring ...]
       python tools/pmc_summary.py profiles/r03e_pmc_raw k_forest   (the committed raw passes)
       python tools/pmc_summary.py --json out.json gpurun_out/pmc_r7   (per-kernel means)
(reads <prefix>a ... <prefix>d directories)
"""
import collections
import csv
import glob
import gzip
import os
import sys


def _passes(prefix):
    """the passes' counter CSVs: rocprofv3 output dirs <prefix>a.. <prefix>d, or a committed
    directory of gzipped passes (profiles/<tag>_pmc_raw/pass_*.csv.gz)"""
    if os.path.isdir(prefix) and glob.glob(os.path.join(prefix, "pass_*.csv.gz")):
        return [gzip.open(f, "rt") for f in sorted(glob.glob(os.path.join(prefix, "pass_*.csv.gz")))]
    return [open(f) for d in sorted(glob.glob(prefix + "*")) for f in glob.glob(d + "/*/*counter_collection.csv")]


def load(prefix):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for fh in _passes(prefix):
        with fh:
            rows = list(csv.DictReader(fh))
            big = collections.defaultdict(int)
            for r in rows:
                big[r["Kernel_Name"]] = max(big[r["Kernel_Name"]], int(r["Grid_Size"]))
            for r in rows:
                if int(r["Grid_Size"]) == big[r["Kernel_Name"]]:
                    per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def to_json(prefix, out):
    """{kernel: {counter: mean, ..., hbm_bytes_per_dispatch}} for bench.py's roofline.traffic"""
    import json

    per = load(prefix)
    res = {}
    for name, ctr in per.items():
        mean = {k: sum(v) / len(v) for k, v in ctr.items()}
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            mean["hbm_bytes_per_dispatch"] = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
        res[name] = mean
    with open(out, "w") as f:
        json.dump({"source": prefix, "correction": "FETCH_SIZE, WRITE_SIZE in KiB; HBM bytes = "
                   "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE reads half of wide streaming "
                   "reads, MI355X_MICROARCH.md HBM section)", "kernels": res}, f, indent=1)


def main():
    if sys.argv[1] == "--json":
        to_json(sys.argv[3], sys.argv[2])
        return
    prefix = sys.argv[1]
    keys = sys.argv[2:] or ["k_forest_chunk", "k_customer", "k_zfill", "k_interleave", "k_terminal"]
    per = load(prefix)
    for name, ctr in per.items():
        if not any(k in name for k in keys):
            continue
        mean = {k: sum(v) / len(v) for k, v in ctr.items()}
        print(name[:90])
        for k in sorted(mean):
            print(f"   {k:24s} {mean[k]:.4g}   (n={len(ctr[k])})")
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            t = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
            print(f"   HBM traffic per dispatch ~ {t / 1e9:.4f} GB (2*FETCH+WRITE)")


if __name__ == "__main__":
    main()
