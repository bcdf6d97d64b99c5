"""Study (tools only): fdx_forest_prepare of configs[2]'s 100M rows as the reference's row-major
[n, 15] float64 X (each lane loads its own 120-B row: ~60 cache lines per load instruction) against
the same values column-major (every load coalesced), alternating; same rank rows required."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from fdx import ops

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    dev = torch.device("cuda", 0)
    arrays, mean, scale, check_X, _ = bench.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    forest = ops.Forest(arrays, 15, mean, scale)
    g = torch.Generator(device=dev)
    g.manual_seed(20240601)
    idx = torch.randint(0, len(check_X), (n,), device=dev, generator=g)
    Xr = torch.from_numpy(check_X).to(dev)[idx]
    Xc = Xr.t().contiguous().t()  # column-major view: strides (1, n)
    ws_r = ops.workspace(forest.workspace_size(n), dev)
    ws_c = ops.workspace(forest.workspace_size(n), dev)
    res = {"row_major": [], "col_major": []}
    for rnd in range(4):
        for name, X, ws in (("row_major", Xr, ws_r), ("col_major", Xc, ws_c)):
            ops.forest_prepare(forest, X, ws)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                ops.forest_prepare(forest, X, ws)
            b.record()
            torch.cuda.synchronize()
            res[name].append(round(a.elapsed_time(b) / 3, 3))
    rows = n * 32  # the rank rows' bytes at the head of the workspace
    same = bool(torch.equal(ws_r[:rows], ws_c[:rows]))
    print(json.dumps({"rows": n, "prepare_ms": res, "rank_rows_equal": same}))


if __name__ == "__main__":
    main()
