"""Study (tools only): does the ORDER of the scoring rows change the forest walk's speed?

The walk is bound by LDS reads (a node read and a rank read per step); node reads of a wave
conflict when its lanes sit on different nodes of one bank (tools/lds_sim.py models it: ~2.5
LDS cycles per node read in the layout's customer-interleaved order, ~2.3 with rows sorted by
their leaves in two trees, ~3.0 random).  This permutes the bench's own rank rows (configs[1],
after FraudPipeline.run_fused) inside the traversal workspace -- sorted by the leaf ids of two
trees (fdx_forest_traverse's leaf output), sorted within 1,024-row tiles only, random -- and
times fdx_forest_traverse on each order; proba is checked bit for bit against the layout order.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    from fdx import _lib, ops, synth
    from fdx.pipeline import FraudPipeline

    dev = torch.device("cuda", 0)
    g = synth.generate_device(50_000, 100_000, 183, seed=1234, device=dev)
    arrays, mean, scale, _, _ = bench.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    forest = ops.Forest(arrays, 15, mean, scale)
    pipe = FraudPipeline(forest=forest)
    n = g["ts"].numel()
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 50_000, 100_000, proba, ws)
    torch.cuda.synchronize()
    m = pipe.last_slots
    z = ws[: 32 * m].view(torch.int16).view(m, 16)  # the rank rows (fdx_forest_traverse's workspace head)
    base = z.clone()

    def timed():
        out = torch.empty(m, dtype=torch.float64, device=dev)
        ops.forest_traverse(forest, m, ws, out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            ops.forest_traverse(forest, m, ws, out)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.reps, out

    ms0, ref = timed()
    # leaf ids of every tree (the general walk with leaf output), for the sort keys
    leaves = torch.empty((m, forest.n_trees), dtype=torch.int32, device=dev)
    buf = torch.empty(m, dtype=torch.float64, device=dev)
    ops.check(_lib.load().fdx_forest_traverse(forest._h, m, ops._ptr(buf), ops._ptr(leaves), ops._ptr(ws), ws.numel(),
                                              None), "fdx_forest_traverse")
    torch.cuda.synchronize()
    l0, l1 = leaves[:, 0].long(), leaves[:, 1].long()
    key2 = l0 * (1 << 20) + l1
    tile = torch.arange(m, device=dev) // 1024
    orders = {
        "layout": torch.arange(m, device=dev),
        "sorted_leaf_t0_t1": torch.argsort(key2, stable=True),
        "tile_sorted_leaf_t0_t1": torch.argsort(tile * (1 << 40) + key2, stable=True),
        "tile_sorted_leaf_t0": torch.argsort(tile * (1 << 40) + l0, stable=True),
        "random": torch.randperm(m, device=dev),
    }
    res = {"layout_first": round(ms0, 4)}
    for name, perm in orders.items():
        z.copy_(base[perm])
        ms, out = timed()
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(m, device=dev)
        res[name] = {"ms": round(ms, 4), "bit_equal": bool(torch.equal(out[inv], ref))}
    z.copy_(base)
    print(json.dumps({"forest_order_ab": res, "slots": m, "chunks": forest.n_chunks}))


if __name__ == "__main__":
    main()
