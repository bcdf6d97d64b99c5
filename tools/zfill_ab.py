"""Study (tools only): where does the row assembly (k_zfill_grouped_w3) spend its time?

configs[1] (50k customers / 100k terminals / 183 days) through FraudPipeline.run_fused with the
slot-order feature table, once per FDX_ZFILL_ORDER value (csrc/fdx_assemble.hip: zfill_order):
0 = the product kernel, 1 / 2 = load-order variants (bit-exact), 4 / 8 / 16 / 32 / 60 = the
kernel with one part of its memory work removed (results NOT the features; timing only).  Run
under `rocprofv3 --kernel-trace --stats`: each variant is its own template instance, so the
stats give its average duration by name.  Prints whether each variant's proba equals variant 0.
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
    ap.add_argument("--orders", default="0,1,2,4,8,16,32,60")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--emit", choices=["slot", "none"], default="slot")
    args = ap.parse_args()
    import torch

    import bench
    from fdx import ops, synth
    from fdx.pipeline import FraudPipeline

    dev = torch.device("cuda", 0)
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, device=dev)
    arrays, mean, scale, _, _ = bench.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    forest = ops.Forest(arrays, 15, mean, scale)
    pipe = FraudPipeline(forest=forest)
    n = g["ts"].numel()
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    rows = ops.FeatureTable(n * 11 // 10, dev) if args.emit == "slot" else None
    a_ = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 50_000, 100_000)
    res, ref = {}, None
    for o in [int(x) for x in args.orders.split(",")]:
        os.environ["FDX_ZFILL_ORDER"] = str(o)
        out = torch.empty(n, dtype=torch.float64, device=dev)
        pipe.run_fused(*a_, out, ws, rows_out=rows)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            pipe.run_fused(*a_, out, ws, rows_out=rows)
        torch.cuda.synchronize()
        res[o] = {"step_ms": round((time.perf_counter() - t0) * 1e3 / args.reps, 3),
                  "proba_equal": bool(torch.equal(out, ref))}
        time.sleep(0.05)
    os.environ.pop("FDX_ZFILL_ORDER")
    print(json.dumps({"zfill_ab": res, "rows": n, "emit": args.emit}))


if __name__ == "__main__":
    main()
