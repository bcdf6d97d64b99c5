"""Headline benchmark: transactions/s featurized + scored, and % of the HBM roofline.

A step = one pass of the hot path over one batch already resident in HBM:
  time flags -> re-key by CUSTOMER_ID -> customer 1/7/30-day windows -> re-key by
  TERMINAL_ID -> terminal delayed-risk windows -> assemble the 15 input_features ->
  StandardScaler + RandomForest(100 trees, depth 20) predict_proba.
Workload per GPU (BASELINE.json configs[1]): 50k customers / 100k terminals / 183 days
(~17.7M tx), synthetic data from the handbook distributions (fdx.synth), scored with the
config-3 model (bench_assets/rf100_d20.npz, trained with sklearn on config-1 features).

N GPUs (torch.distributed.run, one process per GPU): weak scaling, each rank owns its own
50k customers; terminals are shared ids hashed to owner ranks and the terminal half runs
after an RCCL all-to-all re-key (fdx.distributed).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))

METRIC = "transactions/sec featurized+scored (1/2/4/8 GPU) + % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# LDS-issue roofline of the forest walk: a node step = 2 dependent ds_read (node word + the
# row's feature rank), each 2 LDS-array cycles per wave64 instruction (MI355X_MICROARCH.md
# §LDS table, ds_read_b32); one LDS-array cycle per clock per CU, 256 CUs at 2.4 GHz
LDS_PEAK_STEPS = 256 * 2.4e9 / 4 * 64


def walk_steps_per_row(arrays):
    """Steps a row's walks take at most: sum over trees of the tree's max leaf depth (the
    rank walk runs a tree group to its deepest leaf, with a wave-wide early exit every 4 steps
    once all chains sit at leaves -- so this is an upper bound of the executed steps)."""
    import numpy as np

    left, right, off = arrays["left"], arrays["right"], arrays["node_offsets"]
    total = 0
    for t in range(len(off) - 1):
        lo, hi = int(off[t]), int(off[t + 1])
        d = np.zeros(hi - lo, dtype=np.int32)
        lt, rt = left[lo:hi], right[lo:hi]
        for i in range(hi - lo):  # pre-order: a parent precedes its children
            if lt[i] >= 0:
                d[lt[i]] = d[i] + 1
                d[rt[i]] = d[i] + 1
        total += int(d.max())
    return total
# algorithmic bytes per row of the forest launches: every launch reads the row
# (rank layout: 16 x u16 = 32 B; wide layout: 16 x float32 = 64 B), the running float64 sum
# crosses launches (8 B in, 8 B out except the first / last), the last launch writes proba.
RANK_ROW_BYTES, WIDE_ROW_BYTES = 32, 64
# (16 x 4 B slots) in + running float64 sum in + float64 sum/proba out


def forest_bytes_per_row(variant, n_chunks):
    row = RANK_ROW_BYTES if variant >= 16 else WIDE_ROW_BYTES
    return row * n_chunks + 16 * (n_chunks - 1) + 8


def pmc_traffic(variant):
    """HBM bytes per forest launch from the committed rocprofv3 PMC summary
    (profiles/pmc_forest.json, FETCH_SIZE/WRITE_SIZE passes corrected as MI355X_MICROARCH.md
    prescribes) when it was measured on this traversal variant; else (None, None)."""
    p = os.path.join(ROOT, "profiles", "pmc_forest.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    if d.get("variant") != variant:
        return None, None
    return d["hbm_bytes_per_launch"], d["source"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--customers", type=int, default=50_000)
    ap.add_argument("--terminals", type=int, default=100_000)
    ap.add_argument("--days", type=int, default=183)
    ap.add_argument("--model", default=os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-customers", type=int, default=2500)
    ap.add_argument("--breakdown", action="store_true", help="per-stage HIP-event times to stderr")
    ap.add_argument("--slab-rows", type=int, default=0, help="forest traversal slab rows (0 = all rows)")
    ap.add_argument("--sweep-slab", default="", help="comma list of slab sizes to time (stderr)")
    ap.add_argument("--forest-variant", type=int, default=-1,
                    help="traversal kernel shape (fdx_forest_set_variant; -1 = the library default)")
    ap.add_argument("--sweep-variant", default="", help="comma list of forest variants to time (stderr)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU (RCCL all-to-all) path even at 1 GPU (measures its overhead)")
    return ap.parse_args()


def load_model(path):
    import numpy as np

    z = np.load(path)
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    return arrays, z["mean"], z["scale"], z["check_X"], z["check_proba"]


def cpu_baseline(data, arrays, mean, scale, sample_customers):
    """The CPU oracle (C port of the reference's pandas/sklearn arithmetic, 1 thread) on a
    bounded sample: every transaction of customers [0, sample_customers)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle

    m = data["customer"] < sample_customers
    s = {k: v[m] for k, v in data.items()}
    t0 = time.perf_counter()
    f = oracle.featurize_arrays(s["ts"], s["customer"], s["terminal"], s["amount"], s["fraud"])
    names = ["TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + oracle.CUSTOMER_COLS + oracle.TERMINAL_COLS
    X = np.column_stack([s["amount"]] + [f[k] for k in names])
    oracle.forest_predict(X, arrays, mean, scale)
    dt = time.perf_counter() - t0
    return {"value": round(len(s["ts"]) / dt, 1), "unit": "tx/s", "cores": 1, "kind": "port",
            "sample": f"all {len(s['ts'])} tx of customers [0,{sample_customers}) of rank 0's batch: "
                      f"flags + customer/terminal windows + scale + RF(100,d20) predict_proba, "
                      f"C oracle (oracle/fdx_oracle.c), {dt:.1f} s"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from fdx import ops, synth
    from fdx.pipeline import FraudPipeline

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    elif args.sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)

    # weak scaling: every rank adds its own customers and terminals to one shared map
    data = synth.generate(args.customers, args.terminals * world, args.days, seed=1234 + rank,
                          customer_offset=rank * args.customers)
    n_local = len(data["ts"])
    arrays, mean, scale, check_X, check_proba = load_model(args.model)
    forest = ops.Forest(arrays, 15, mean, scale)
    forest.set_slab_rows(args.slab_rows)
    default_variant = forest.variant
    if args.forest_variant >= 0:
        forest.set_variant(args.forest_variant)
    T = lambda a, d: torch.from_numpy(np.ascontiguousarray(a)).to(dev, d)  # noqa: E731
    # sanity: the GPU forest reproduces sklearn on the held-out sample saved with the model
    got = forest.predict(T(check_X, torch.float64)).cpu().numpy()
    if not np.array_equal(got, check_proba):
        raise SystemExit("forest parity check against sklearn failed")

    ts, cust, term = T(data["ts"], torch.int64), T(data["customer"], torch.int32), T(data["terminal"], torch.int32)
    amt, fr = T(data["amount"], torch.float64), T(data["fraud"], torch.uint8)
    pipe = FraudPipeline(forest=forest)
    ws = ops.workspace(forest.workspace_size(n_local * 11 // 10), dev)  # scoring slots incl. layout padding
    proba = torch.empty(n_local, dtype=torch.float64, device=dev)
    ev = []

    if world > 1 or args.sharded:
        from fdx.distributed import ShardedPipeline

        sp = ShardedPipeline(pipe, world, rank, args.terminals * world)
        n_cust_total = args.customers * world

        def step(record):
            sp.run(ts, cust, term, amt, fr, n_cust_total, proba, ws, ev if record else None)

        if rank == 0:
            print(f"rank0 tx={n_local}", file=sys.stderr)
    else:
        def step(record):
            marks = []

            def mark(i):
                if record:
                    e = torch.cuda.Event(enable_timing=True)
                    e.record()
                    marks.append(e)

            pipe.run_fused(ts, cust, term, amt, fr, args.customers, args.terminals, proba, ws, on_traverse=mark)
            if record:
                ev.append(tuple(marks))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt, float(n_local)], dtype=torch.float64, device=dev)
        dtm = t[:1].clone()
        dist.all_reduce(dtm, op=dist.ReduceOp.MAX)
        tot = t[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dt, n_total = float(dtm.item()), int(tot.item())
    else:
        n_total = n_local

    trav_ms = sum(a.elapsed_time(b) for a, b in ev) / max(len(ev), 1)
    slab = args.slab_rows if args.slab_rows > 0 else n_local
    launches = forest.n_chunks * -(-n_local // slab)
    launch_ms = trav_ms / launches
    # every launch streams its slab's rows once: total algorithmic bytes / total time
    fvar = forest.variant if args.forest_variant < 0 else args.forest_variant
    bpr = forest_bytes_per_row(fvar, forest.n_chunks)
    achieved = bpr * n_local / (trav_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(fvar)
    out = {
        "metric": METRIC,
        "value": round(n_total * args.steps / dt, 1),
        "unit": "tx/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: handbook-distribution generator (fdx.synth, seed 1234+rank), resident in HBM",
        "config": {"workload": f"configs[1]: {args.customers} customers / {args.terminals} terminals / "
                               f"{args.days} days per GPU, featurize + RF(100 trees, depth 20) predict_proba",
                   "tx_per_gpu": n_local, "global_tx": n_total, "parallelism": f"customer-sharded x{world}",
                   "model": "bench_assets/rf100_d20.npz (sklearn RandomForest, config-1 features)"},
        "roofline": {"kernel": "k_forest_rank" if fvar >= 16 else "k_forest_chunk", "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_unit": "bytes per launch",
                     "algorithmic_bytes_per_launch": round(bpr / forest.n_chunks * n_local),
                     "traffic_source": traffic_src, "avg_launch_ms": round(launch_ms, 4),
                     "launches_per_step": launches,
                     "traverse_ms": round(trav_ms, 3),
                     "forest_variant": fvar,
                     "bytes_per_row_per_launch": round(bpr / forest.n_chunks, 2)},
    }
    steps = walk_steps_per_row(arrays)
    ach_steps = steps * n_local / (trav_ms * 1e-3)
    out["roofline_lds"] = {"kernel": out["roofline"]["kernel"], "bound": "lds", "unit": "node steps/s",
                           "achieved": float(f"{ach_steps:.4g}"), "peak": float(f"{LDS_PEAK_STEPS:.4g}"),
                           "frac": round(ach_steps / LDS_PEAK_STEPS, 4), "node_steps_per_row_max": steps,
                           "note": "2 ds_read per step at 2 LDS cycles each; steps = sum of tree depths (upper "
                                   "bound: wave-wide early exit), so frac is an upper bound"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(data, arrays, mean, scale, args.cpu_sample_customers)
    if args.sweep_slab and rank == 0:
        res = {}
        for sr in [int(x) for x in args.sweep_slab.split(",")]:
            forest.set_slab_rows(sr)
            ops.forest_traverse(forest, n_local, ws, proba)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                ops.forest_traverse(forest, n_local, ws, proba)
            b.record()
            torch.cuda.synchronize()
            res[sr] = round(a.elapsed_time(b) / 3, 3)
        forest.set_slab_rows(args.slab_rows)
        print(json.dumps({"slab_sweep_traverse_ms": res}), file=sys.stderr)
    if args.sweep_variant and rank == 0:
        # each variant: one full untimed pipeline pass (the prepared row format depends on
        # the layout), bit-equality of proba against the default, then 3 timed traversals
        res = {}
        ref = proba.clone()
        for v in [int(x) for x in args.sweep_variant.split(",")]:
            forest.set_variant(v)
            pv = torch.empty_like(proba)
            pipe.run_fused(ts, cust, term, amt, fr, args.customers, args.terminals, pv, ws)
            same = bool(torch.equal(pv, ref))
            wsv, n_rows = pipe._forest_ws(pipe.last_slots, ws, dev), pipe.last_slots
            buf = torch.empty(n_rows, dtype=torch.float64, device=dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                ops.forest_traverse(forest, n_rows, wsv, buf)
            b.record()
            torch.cuda.synchronize()
            res[v] = {"ms": round(a.elapsed_time(b) / 3, 3), "chunks": forest.n_chunks, "bit_equal": same}
        forest.set_variant(args.forest_variant if args.forest_variant >= 0 else default_variant)
        print(json.dumps({"variant_sweep_traverse": res}), file=sys.stderr)
    if args.breakdown and rank == 0:
        print(json.dumps(stage_breakdown(pipe, forest, ts, cust, term, amt, fr, args, ws, proba)),
              file=sys.stderr)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1 or args.sharded:
        dist.destroy_process_group()


def stage_breakdown(pipe, forest, ts, cust, term, amt, fr, args, ws, proba):
    import torch

    from fdx import ops

    marks = []

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((name, e))

    n = ts.numel()
    mark("start")
    cperm, cseg, _ = ops.rekey(cust, args.customers)
    mark("rekey_customer")
    lay = ops.customer_layout(cseg, cperm, ts, amt, 3, windows_days=(1, 7, 30))
    mark("customer_layout")
    inb, isum = ops.customer_windows_walk(lay, cseg)
    mark("customer_windows")
    tperm, tseg, _ = ops.rekey(term, args.terminals)
    mark("rekey_terminal")
    trec = ops.terminal_windows_packed(ts, fr, tseg, rows=tperm)
    mark("terminal_windows")
    wsb = pipe._forest_ws(lay.n_slots, ws, ts.device)
    ops.forest_prepare_grouped(forest, 0, lay.its, lay.iamt, inb, isum, lay.irow, None, trec, wsb, n=lay.n_slots,
                               val_is_sum=True)
    mark("assemble_scale_z32")
    ops.forest_traverse_perm(forest, lay.n_slots, wsb, proba, lay.irow)
    mark("forest_traverse")
    torch.cuda.synchronize()
    return {"breakdown_ms": {marks[i][0]: round(marks[i - 1][1].elapsed_time(marks[i][1]), 4)
                             for i in range(1, len(marks))}, "n": n, "scoring_slots": lay.n_slots}


if __name__ == "__main__":
    main()
