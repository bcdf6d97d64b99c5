"""BASELINE.json configs[2]: RandomForest(100 trees, depth 20) predict_proba over 100M feature
rows on one MI355X (the reference's scoring call, model.predict_proba(scaler.transform(X))[:, 1],
fraud_detection.py:190-193 / model_training.ipynb:506).

Rows: the bench model's 4,096 held-out config-1 feature rows (bench_assets/rf100_d20.npz,
sklearn predict_proba saved beside them) resampled with a fixed seed to --rows rows, resident
in HBM as the float64 [n, 15] matrix the reference passes.  A step = fdx_forest_prepare
(scale + float32 cast + threshold ranks) + fdx_forest_traverse over all rows.  Every sampled
row's probability must equal sklearn's bit for bit (checked on the full output after timing).
Prints one JSON line (rows/s, per-stage ms, HBM and LDS rooflines).

--model bench_assets/rf_deployed.npz: the reference's DEPLOYED model instead --
RandomForestClassifier(random_state=0), 100 unlimited-depth trees, 1.68M nodes
(model_training.ipynb:2212, served at fraud_detection.py:81-82), rebuilt in the build container
(bench_assets/make_deployed.py) -- on the rows of the notebook's own test set (66,452 rows,
sklearn's predict_proba saved beside them).  Besides the resampled throughput, the line then
carries "reference_call": the notebook's timed call itself (predict_proba of those 66,452
rows, model_training.ipynb:2524-2525: 0.476645 s = 139,414 rows/s on the authors' CPU) as
one prepare + traverse on HBM-resident rows, and with the host copy in and out."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default=os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    ap.add_argument("--variant", type=int, default=-1, help="forest walk variant (fdx.h; -1: the library's choice)")
    ap.add_argument("--range-rows", type=int, default=-1, help="rows per traversal range (-1: the library's choice)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fdx import ops

    dev = torch.device("cuda", 0)
    z = np.load(args.model)
    deployed = "test_X" in z.files
    if deployed:
        arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
                  for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
        mean, scale, check_X, check_proba = z["mean"], z["scale"], z["test_X"], z["test_proba1"]
    else:
        arrays, mean, scale, check_X, check_proba = bench.load_model(args.model)
    forest = ops.Forest(arrays, 15, mean, scale)
    if args.variant >= 0:
        forest.set_variant(args.variant)
    if args.range_rows >= 0:
        forest.set_range_rows(args.range_rows)
    n = args.rows
    g = torch.Generator(device=dev)
    g.manual_seed(20240601)
    idx = torch.randint(0, len(check_X), (n,), device=dev, generator=g)
    X = torch.from_numpy(check_X).to(dev)[idx]  # [n, 15] float64, 120 B per row
    ws = ops.workspace(forest.workspace_size(n), dev)
    out = torch.empty(n, dtype=torch.float64, device=dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        ops.forest_prepare(forest, X, ws)
        if ev is not None:
            ev[1].record()
        ops.forest_traverse(forest, n, ws, out)
        if ev is not None:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e in evs:
        step(e)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prep_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    trav_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    exp = torch.from_numpy(check_proba).to(dev)[idx]
    if not torch.equal(out, exp):
        raise SystemExit(f"predict_proba differs from sklearn on {int((out != exp).sum())} of {n} rows")
    ref_call = None
    if deployed:  # the notebook's timed call: predict_proba of the 66,452 test rows
        m = len(check_X)
        Xh = torch.from_numpy(np.ascontiguousarray(check_X)).pin_memory()
        Xm = Xh.to(dev)
        wsm = ops.workspace(forest.workspace_size(m), dev)
        om = torch.empty(m, dtype=torch.float64, device=dev)
        oh = torch.empty(m, dtype=torch.float64).pin_memory()
        reps = 20
        for host in (False, True):
            for r in range(reps + 2):  # 2 untimed
                if r == 2:
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                if host:
                    Xm.copy_(Xh, non_blocking=True)
                ops.forest_prepare(forest, Xm, wsm)
                ops.forest_traverse(forest, m, wsm, om)
                if host:
                    oh.copy_(om, non_blocking=True)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t1) / reps * 1e3
            if host:
                ref_call["host_in_out_ms"] = round(ms, 3)
            else:
                ref_call = {"rows": m, "ms": round(ms, 3), "rows_per_s": round(m / ms * 1e3, 1),
                            "published_s": 0.476645, "published_rows_per_s": 139414,
                            "vs_published": round(m / ms * 1e3 / 139414, 1)}
        if not torch.equal(om, torch.from_numpy(check_proba).to(dev)):
            raise SystemExit("deployed model: predict_proba of the test set differs from sklearn")
    steps_row = bench.walk_steps_per_row(arrays)
    lds = steps_row * n / (trav_ms * 1e-3)
    prep_gbs = n * (120 + 32) / (prep_ms * 1e-3) / 1e9  # f64 row in, u16 rank row out
    line = {
        "metric": ("deployed RF(100, unlimited depth) predict_proba rows/s on one MI355X" if deployed else
                   "configs[2]: RF(100, depth 20) predict_proba rows/s on one MI355X"),
        "value": round(n * args.steps / dt, 1), "unit": "rows/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "dtype": "f64 in, f32 compare (sklearn's), f64 accumulate", "rows": n,
        "variant": forest.variant,
        "data": ("the notebook test set's 66,452 rows" if deployed else "bench model's 4,096 held-out config-1 feature rows")
        + " resampled (seed 20240601), resident in HBM",
        "bit_exact_vs_sklearn": True, "prepare_ms": round(prep_ms, 3), "traverse_ms": round(trav_ms, 3),
        "roofline_prepare": {"bound": "hbm", "achieved": round(prep_gbs, 1), "peak": bench.HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(prep_gbs / bench.HBM_PEAK_GBS, 4),
                             "bytes_per_row": 152},
        "roofline_lds": {"bound": "lds", "unit": "node steps/s", "achieved": float(f"{lds:.4g}"),
                         "peak": float(f"{bench.LDS_PEAK_STEPS:.4g}"), "frac": round(lds / bench.LDS_PEAK_STEPS, 4),
                         "node_steps_per_row_max": steps_row},
    }
    if ref_call is not None:
        line["reference_call"] = ref_call
    print(json.dumps(line))


if __name__ == "__main__":
    main()
