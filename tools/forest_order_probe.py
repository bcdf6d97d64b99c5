"""Probe: how much does the ORDER of the scoring rows change the forest walk's time?

Lanes of a wave walk the same tree at the same step; when their rows take the same path, the
node reads broadcast (one LDS address) and the wave-wide early exit triggers together.  This
probe builds the bench's rank rows (config-2 workload, fused pipeline), then times
fdx_forest_traverse over the same rows in several orders (each checked against the
original order's probabilities, permuted):
  identity   -- the layout's slot order (what the pipeline scores)
  shuffled   -- a random permutation (no locality at all)
  amount     -- sorted by the rank of feature 0 (TX_AMOUNT)
  leaf0      -- sorted by the leaf each row reaches in tree 0
  leaf01     -- sorted by (leaf in tree 0, leaf in tree 1)
  same       -- every row = row 0 (all walks identical: the broadcast bound)
Prints one JSON line to stdout.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)


def main():
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
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"], 50_000, 100_000, proba, ws)
    torch.cuda.synchronize()
    m = pipe.last_slots
    z = ws[: m * 32].view(torch.int16).view(m, 16)
    base = ws.clone()
    ref = torch.empty(m, dtype=torch.float64, device=dev)
    ops.forest_traverse(forest, m, base, ref)
    leaves = torch.empty((m, forest.n_trees), dtype=torch.int32, device=dev)
    from fdx import _lib
    L = _lib.load()
    _lib.check(L.fdx_forest_traverse(forest._h, m, ops._ptr(torch.empty(m, dtype=torch.float64, device=dev)),
                                     ops._ptr(leaves), ops._ptr(base), base.numel(), ops._s(None)), "traverse")
    torch.cuda.synchronize()
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    orders = {
        "identity": torch.arange(m, device=dev),
        "shuffled": torch.randperm(m, device=dev, generator=gen),
        "amount": torch.argsort(z[:, 0].to(torch.int32) & 0xFFFF, stable=True),
        "leaf0": torch.argsort(leaves[:, 0].long(), stable=True),
        "leaf01": torch.argsort(leaves[:, 0].long() * (1 << 20) + leaves[:, 1].long(), stable=True),
        "same": torch.zeros(m, dtype=torch.int64, device=dev),
    }
    res = {"rows": m, "chunks": forest.n_chunks}
    for name, o in orders.items():
        w2 = base.clone()
        w2[: m * 32].view(torch.int16).view(m, 16).copy_(z[o])
        out = torch.empty(m, dtype=torch.float64, device=dev)
        ops.forest_traverse(forest, m, w2, out)  # warm
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            ops.forest_traverse(forest, m, w2, out)
        b.record()
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, ref[o]))
        res[name] = {"ms": round(a.elapsed_time(b) / 3, 3), "bit_equal": ok}
        print(name, res[name], file=sys.stderr, flush=True)
    print(json.dumps({"forest_order_probe": res}))


if __name__ == "__main__":
    main()
