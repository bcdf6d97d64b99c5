"""BASELINE.json configs[2]: RandomForest(100 trees, depth 20) predict_proba over 100M feature
rows on one MI355X (the reference's scoring call, model.predict_proba(scaler.transform(X))[:, 1],
fraud_detection.py:190-193 / model_training.ipynb:506).

Rows: the bench model's 4,096 held-out config-1 feature rows (bench_assets/rf100_d20.npz,
sklearn predict_proba saved beside them) resampled with a fixed seed to --rows rows, resident
in HBM as the float64 [n, 15] matrix the reference passes.  A step = fdx_forest_prepare
(scale + float32 cast + threshold ranks) + fdx_forest_traverse over all rows.  Every sampled
row's probability must equal sklearn's bit for bit (checked on the full output after timing).
Prints one JSON line (rows/s, per-stage ms, HBM and LDS rooflines)."""
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
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fdx import ops

    dev = torch.device("cuda", 0)
    arrays, mean, scale, check_X, check_proba = bench.load_model(args.model)
    forest = ops.Forest(arrays, 15, mean, scale)
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
    steps_row = bench.walk_steps_per_row(arrays)
    lds = steps_row * n / (trav_ms * 1e-3)
    prep_gbs = n * (120 + 32) / (prep_ms * 1e-3) / 1e9  # f64 row in, u16 rank row out
    print(json.dumps({
        "metric": "configs[2]: RF(100, depth 20) predict_proba rows/s on one MI355X",
        "value": round(n * args.steps / dt, 1), "unit": "rows/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "dtype": "f64 in, f32 compare (sklearn's), f64 accumulate", "rows": n,
        "data": "bench model's 4,096 held-out config-1 feature rows resampled (seed 20240601), resident in HBM",
        "bit_exact_vs_sklearn": True, "prepare_ms": round(prep_ms, 3), "traverse_ms": round(trav_ms, 3),
        "roofline_prepare": {"bound": "hbm", "achieved": round(prep_gbs, 1), "peak": bench.HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(prep_gbs / bench.HBM_PEAK_GBS, 4),
                             "bytes_per_row": 152},
        "roofline_lds": {"bound": "lds", "unit": "node steps/s", "achieved": float(f"{lds:.4g}"),
                         "peak": float(f"{bench.LDS_PEAK_STEPS:.4g}"), "frac": round(lds / bench.LDS_PEAK_STEPS, 4),
                         "node_steps_per_row_max": steps_row},
    }))


if __name__ == "__main__":
    main()
