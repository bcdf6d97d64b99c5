"""A/B of FraudPipeline class switches on one box, alternating (tools only): the bench's step
(configs[1], run_fused with the featurized table) timed as --steps steps per round, the settings
alternating for --rounds rounds; prints the per-round ms/step of each setting and their medians.
    python tools/step_ab.py tail_on_side=1 tail_on_side=0 [--rounds 6 --steps 10]
A setting is attr=value on FraudPipeline (ints)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("settings", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fdx import ops, synth
    from fdx.pipeline import FraudPipeline

    dev = torch.device("cuda", 0)
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, device=dev)
    n = g["ts"].numel()
    arrays, mean, scale, _, _ = bench.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    forest = ops.Forest(arrays, 15, mean, scale)
    pipe = FraudPipeline(forest=forest)
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    rows = ops.FeatureTable(n * 11 // 10, dev)
    args_ = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 50_000, 100_000, proba, ws)
    parsed = []
    for s in args.settings:
        parsed.append({kv.split("=")[0]: (float if "." in kv.split("=")[1] else int)(kv.split("=")[1])
                       for kv in s.split(",")})
    ref = None
    res = {s: [] for s in args.settings}
    for rnd in range(args.rounds):
        for s, kv in zip(args.settings, parsed):
            for k, v in kv.items():
                setattr(FraudPipeline, k, v)
            for _ in range(3):
                pipe.run_fused(*args_, rows_out=rows)
            torch.cuda.synchronize()
            if ref is None:
                ref = proba.clone()
            assert torch.equal(proba, ref), s
            t0 = time.perf_counter()
            for _ in range(args.steps):
                pipe.run_fused(*args_, rows_out=rows)
            torch.cuda.synchronize()
            res[s].append((time.perf_counter() - t0) / args.steps * 1e3)
    out = {s: {"ms_per_step": [round(x, 3) for x in v], "median": round(float(np.median(v)), 3)} for s, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
