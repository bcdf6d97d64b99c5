"""A/B probe for the forest traversal on the bench's own scoring rows: configs[1] (50k
customers / 100k terminals / 183 days) featurized by FraudPipeline.run_fused, then for each
forest variant (fdx_forest_set_variant) the traversal of the step's scoring rows (fdx_forest_traverse
over the slots, proba by slot) timed alone, --reps times after one untimed call, with the
probabilities checked bit for bit against the default variant.  Run under
`rocprofv3 --kernel-trace` to get per-launch durations (variants are separated by a 50 ms idle
gap; each prints its chunk count).  Tools only.
"""
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
    ap.add_argument("--variants", default="1")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch

    import bench
    from fdx import ops, synth
    from fdx.pipeline import FraudPipeline

    dev = torch.device("cuda", 0)
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, device=dev)
    arrays, mean, scale, _, _ = bench.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    forest = ops.Forest(arrays, 15, mean, scale)
    default = forest.variant
    pipe = FraudPipeline(forest=forest)
    n = g["ts"].numel()
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    ref = torch.empty(n, dtype=torch.float64, device=dev)
    args_ = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 50_000, 100_000)
    pipe.run_fused(*args_, ref, ws)
    torch.cuda.synchronize()
    res = {}
    for rnd in range(args.rounds):
        for v in [int(x) for x in args.variants.split(",")]:
            forest.set_variant(v)
            pv = torch.empty_like(ref)
            pipe.run_fused(*args_, pv, ws)  # the rows in this variant's format
            torch.cuda.synchronize()
            time.sleep(0.05)
            m = pipe.last_slots
            buf = torch.empty(m, dtype=torch.float64, device=dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ops.forest_traverse(forest, m, ws, buf)
            a.record()
            for _ in range(args.reps):
                ops.forest_traverse(forest, m, ws, buf)
            b.record()
            torch.cuda.synchronize()
            r = res.setdefault(v, {"ms": [], "chunks": forest.n_chunks, "bit_equal": True})
            r["ms"].append(round(a.elapsed_time(b) / args.reps, 4))
            r["bit_equal"] = r["bit_equal"] and bool(torch.equal(pv, ref))
            time.sleep(0.05)
    forest.set_variant(default)
    print(json.dumps({"forest_ab": res, "rows": n, "slots": pipe.last_slots}))


if __name__ == "__main__":
    main()
