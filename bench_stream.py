"""Config 5 benchmark (BASELINE.json configs[4]): streaming micro-batches of 64k CDC
transactions -- incremental customer / terminal window state update + StandardScaler +
RandomForest(100, depth 20) predict_proba -- p50 / p99 batch latency.

Workload: the tail of config 4 (1M customers / 2M terminals, handbook distributions,
fdx.synth).  History: --history-days days streamed into the state first (day-sized batches,
untimed), so every ring holds a realistic 30 / 37-day window; then the next day is cut into
micro-batches of --batch transactions (global) and each is timed end to end:
  host batch (pinned) -> HBM -> fdx_stream_update (2 launches) -> forest -> proba -> host.
Also reported: the device-only time of the update + scoring (HIP events) and the rate.

N GPUs, one process per GPU (torch.distributed.run, or `--gpus N` alone: the script starts
the N ranks itself, bench.spawn_ranks): customers sharded by contiguous id
range, each micro-batch split by customer owner, terminals owned by id % N, one RCCL
all-to-all there and back per batch (fdx.streaming.ShardedStreamScorer); the batch latency
is the max over ranks.  Rank 0 prints one JSON line.

usage: python bench_stream.py [--gpus N] [--batches K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "real-time_fraud_detection_system_amd"))


def cdc_encode(tx_id, customer, terminal, amount, ts_ns, kafka_ts, dup_frac=0.0, seed=0):
    """The Debezium wire columns of a batch of transactions, as the reference's sink receives
    them (pyspark/scripts/kafka_s3_sink_transactions.py:77-126): tx_amount DECIMAL(10,2) as
    big-endian two's-complement bytes of the cents (minimal length, as Kafka Connect encodes
    it), tx_datetime in microseconds, ids int64, a Kafka timestamp per record.  dup_frac adds,
    for that fraction of the records, a STALE update of the same tx_id (older Kafka timestamp,
    another amount) placed earlier or later in the batch -- the dedup (:180) must drop it.
    -> dict of numpy arrays (blob uint8 + offsets int64 [n' + 1]) with n' >= n records."""
    import numpy as np

    n = len(tx_id)
    cents = np.rint(np.asarray(amount, np.float64) * 100.0).astype(np.int64)
    rec = {"tx_id": np.asarray(tx_id, np.int64), "customer": np.asarray(customer, np.int64),
           "terminal": np.asarray(terminal, np.int64), "cents": cents,
           "us": np.asarray(ts_ns, np.int64) // 1000, "kts": np.asarray(kafka_ts, np.int64)}
    if dup_frac > 0 and n:
        rng = np.random.default_rng(seed)
        d = rng.choice(n, max(1, int(n * dup_frac)), replace=False)
        stale = {k: v[d].copy() for k, v in rec.items()}
        stale["cents"] = stale["cents"] + rng.integers(1, 10_000, len(d))
        stale["kts"] = stale["kts"] - rng.integers(1, 1000, len(d))
        pos = rng.integers(0, n + 1, len(d))      # insertion points in the batch
        order = np.argsort(np.r_[np.arange(n) * 2 + 1, pos * 2], kind="stable")
        rec = {k: np.r_[rec[k], stale[k]][order] for k in rec}
    c = rec["cents"]
    nbytes = np.maximum(1, (_bit_length(c) + 8) // 8)
    offsets = np.r_[0, np.cumsum(nbytes)].astype(np.int64)
    blob = np.zeros(int(offsets[-1]), np.uint8)
    u = c.astype(np.uint64)  # two's complement bits
    for k in range(8):  # byte k from the END of each record: (u >> 8k) & 0xFF
        m = nbytes > k
        blob[offsets[1:][m] - 1 - k] = ((u[m] >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    return {"tx_id": rec["tx_id"], "customer": rec["customer"], "terminal": rec["terminal"], "blob": blob,
            "offsets": offsets, "us": rec["us"], "kts": rec["kts"], "cents": c}


def _bit_length(c):
    """int.bit_length of the two's-complement magnitude: v >= 0 -> bits of v, v < 0 -> bits of ~v."""
    import numpy as np

    m = np.where(c < 0, ~c, c).astype(np.uint64)
    bl = np.zeros(len(m), np.int64)
    for s in range(63, -1, -1):
        hit = (bl == 0) & ((m >> np.uint64(s)) != 0)
        bl[hit] = s + 1
    return bl


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="as bench.py: every rank on cuda:0, gloo, host-staged exchange collectives (not a measurement)")
    ap.add_argument("--customers", type=int, default=1_000_000)
    ap.add_argument("--terminals", type=int, default=2_000_000)
    ap.add_argument("--history-days", type=int, default=38)
    ap.add_argument("--batch", type=int, default=65536, help="global transactions per micro-batch")
    ap.add_argument("--batches", type=int, default=0, help="timed batches (0 = the whole streamed day)")
    ap.add_argument("--warmup", type=int, default=3, help="untimed micro-batches before the timed ones")
    ap.add_argument("--customer-ring", type=int, default=256)
    ap.add_argument("--terminal-ring", type=int, default=256)
    ap.add_argument("--model", default=os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    ap.add_argument("--column-copies", action="store_true",
                    help="a batch's 5 columns copied to the device one by one (default: one packed pinned buffer)")
    ap.add_argument("--no-graph", action="store_true",
                    help="enqueue each batch's kernels one by one (default at world 1: one HIP graph per batch "
                         "size, StreamScorer.score_graph, the probabilities' copy to the host inside it)")
    ap.add_argument("--cdc", action="store_true",
                    help="timed batches arrive as Debezium wire columns (decimal bytes, us timestamps, Kafka "
                         "timestamps, 2%% stale duplicate updates): device decode + dedup + compact + score "
                         "(StreamScorer.score_cdc; world 1)")
    return ap.parse_args(argv)


def rank_shard(args, world: int, rank: int):
    """configs[4]'s key state over the ranks: rank r owns the contiguous customer ids
    [r * n_c, (r + 1) * n_c) (n_c = customers // world) and all terminals (terminal t is owned
    by t % world for the exchange).  Returns (n_c, customer_base, n_terminals)."""
    n_c = args.customers // world
    return n_c, rank * n_c, args.terminals


def main():
    args = parse()
    from bench import load_model, rehearse_host_collectives, spawn_ranks, stdout_to_stderr

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))  # one process per GPU, before this one touches the GPU
    json_out = stdout_to_stderr()
    import numpy as np
    import torch
    import torch.distributed as dist

    from fdx import ops, synth
    from fdx.streaming import ShardedStreamScorer, StreamScorer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    cdev = torch.device("cpu") if args.rehearse_one_gpu else dev  # this script's own collectives
    if world > 1 and args.rehearse_one_gpu:
        dist.init_process_group("gloo")
        rehearse_host_collectives()
    elif world > 1:
        dist.init_process_group("nccl", device_id=dev)

    n_c, base, _ = rank_shard(args, world, rank)
    t_gen = time.perf_counter()
    # generated on the GPU (csrc/fdx_synth.hip), then copied to host: the micro-batches arrive
    # from pinned host memory, as CDC batches would
    # one population for every N (draws keyed by the global customer id): the union of the ranks'
    # rows is the same stream at every world size
    g = synth.generate_device(n_c, args.terminals, args.history_days + 1, seed=4321, customer_offset=base,
                              n_customers_total=n_c * world, device=dev)
    d = {k: g[k].cpu().numpy() for k in ("ts", "customer", "terminal", "amount", "fraud")}
    del g
    t_gen = time.perf_counter() - t_gen
    split = synth.START_NS + args.history_days * 86400 * synth.NS
    h = int(np.searchsorted(d["ts"], split))
    day_ns = 86400 * synth.NS

    arrays, mean, scale, check_X, check_proba = load_model(args.model)
    forest = ops.Forest(arrays, 15, mean, scale)
    T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
    if not np.array_equal(forest.predict(T(check_X, torch.float64)).cpu().numpy(), check_proba):
        raise SystemExit("forest parity check against sklearn failed")

    # history batches: one per day (untimed); the state's batch capacity covers them
    day_cuts = np.searchsorted(d["ts"][:h], synth.START_NS + np.arange(args.history_days + 1) * day_ns)
    max_day = int(np.diff(day_cuts).max()) if h else 0
    per_rank = args.batch // world
    # common micro-batch time cuts: every per_rank-th timestamp of rank 0's streamed day
    s_ts = d["ts"][h:]
    if rank == 0:
        cuts = s_ts[::per_rank].astype(np.int64)
        cuts = np.r_[cuts, s_ts[-1] + 1] if len(s_ts) else np.array([split, split + 1])
        hdr = torch.tensor([len(cuts)], dtype=torch.int64, device=cdev)
    else:
        hdr = torch.zeros(1, dtype=torch.int64, device=cdev)
    if world > 1:
        dist.broadcast(hdr, 0)
    cut_t = torch.zeros(int(hdr.item()), dtype=torch.int64, device=cdev)
    if rank == 0:
        cut_t.copy_(torch.from_numpy(cuts))
    if world > 1:
        dist.broadcast(cut_t, 0)
    cuts = cut_t.cpu().numpy()
    bounds = np.searchsorted(s_ts, cuts) + h
    bounds[0], bounds[-1] = h, len(d["ts"])
    max_mb = int(np.diff(bounds).max())
    cap = max(max_day, max_mb, 1)

    wire = None
    if args.cdc:
        if world > 1:
            raise SystemExit("--cdc runs at world 1 (StreamScorer.score_cdc)")
        # the streamed day as CDC micro-batches, encoded up front (untimed): pinned host
        # buffers per batch, as a Kafka consumer would hold them
        kts = np.arange(len(d["ts"]), dtype=np.int64) * 10 + 1_739_000_000_000
        wire = []
        for k in range(len(bounds) - 1):
            a, b = int(bounds[k]), int(bounds[k + 1])
            r = cdc_encode(np.arange(a, b), d["customer"][a:b], d["terminal"][a:b], d["amount"][a:b], d["ts"][a:b],
                           kts[a:b], dup_frac=0.02, seed=k)
            wire.append({key: torch.from_numpy(np.ascontiguousarray(r[key] if len(r[key]) else np.zeros(1, r[key].dtype)))
                         .pin_memory() for key in ("tx_id", "customer", "terminal", "blob", "offsets", "us", "kts")})
        cap_w = max(int(w["tx_id"].numel()) for w in wire)
        cap = max(cap, cap_w)
        wdev = {key: torch.empty(max(int(w[key].numel()) for w in wire), dtype=wire[0][key].dtype, device=dev)
                for key in wire[0]}

    if world > 1:
        sc = ShardedStreamScorer(forest, world, rank, n_c, base, args.terminals, customer_ring=args.customer_ring,
                                 terminal_ring=args.terminal_ring, max_batch=cap, max_recv=cap * world * 2)
    else:
        sc = StreamScorer(forest, n_c, args.terminals, customer_ring=args.customer_ring,
                          terminal_ring=args.terminal_ring, max_batch=cap)
    cols = [("ts", torch.int64), ("customer", torch.int32), ("amount", torch.float64), ("terminal", torch.int32),
            ("fraud", torch.uint8)]
    # pinned host copies of the whole input (the "arriving" micro-batches are slices)
    pin = {k: torch.from_numpy(np.ascontiguousarray(d[k])).pin_memory() for k, _ in cols}
    dcols = {k: torch.empty(cap, dtype=t, device=dev) for k, t in cols}
    out_h = torch.empty(cap, dtype=torch.float64).pin_memory()

    def run_cdc(k, ev=None):
        w = wire[k]
        n = int(w["tx_id"].numel())
        for key, t in w.items():
            wdev[key][:t.numel()].copy_(t, non_blocking=True)
        if ev is not None:
            ev[0].record()
        p, rows = sc.score_cdc(wdev["tx_id"][:n], wdev["customer"][:n], wdev["terminal"][:n],
                               wdev["blob"][:int(w["blob"].numel())], wdev["offsets"][:n + 1], wdev["us"][:n],
                               wdev["kts"][:n])
        if ev is not None:
            ev[1].record()
        m = p.numel()
        out_h[:m].copy_(p, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return m

    # a streamed micro-batch arrives as ONE pinned host buffer holding its 5 columns back to back
    # (ts 8n | amount 8n | customer 4n | terminal 4n | fraud n bytes: every column aligned), as a
    # consumer would fill it -- one host-to-device copy instead of five (each copy costs ~9 us of
    # enqueue gap: 100 -> ~35 us per 64k batch, profiles/r06e trace); packed up front, untimed
    packed_cols = [("ts", torch.int64, 8), ("amount", torch.float64, 8), ("customer", torch.int32, 4),
                   ("terminal", torch.int32, 4), ("fraud", torch.uint8, 1)]
    dstage = torch.empty(25 * cap, dtype=torch.uint8, device=dev)

    def pack(a, b):
        buf = torch.empty(25 * (b - a), dtype=torch.uint8).pin_memory()
        o = 0
        for k, _, w in packed_cols:
            buf[o:o + w * (b - a)].copy_(pin[k][a:b].view(torch.uint8))
            o += w * (b - a)
        return buf

    def stage_views(n):
        views, o = {}, 0
        for key, t, w in packed_cols:
            views[key] = dstage[o:o + w * n].view(t)
            o += w * n
        return [views[key] for key, _ in cols]

    # one HIP graph per batch size (world 1): the batch's ~10 launches + the probabilities' copy
    # to the host as one graph launch; every size of the streamed day is captured before the
    # first timed batch (a consumer of fixed-size batches captures once)
    graph = world == 1 and not args.no_graph

    def run_packed(k, ev=None):
        buf = packed[k]
        n = buf.numel() // 25
        dstage[:25 * n].copy_(buf, non_blocking=True)
        if ev is not None:
            ev[0].record()
        if graph:
            sc.score_graph(*stage_views(n), out_host=out_h)
            if ev is not None:
                ev[1].record()
        else:
            p = sc.score(*stage_views(n))
            if ev is not None:
                ev[1].record()
            out_h[:n].copy_(p, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return n

    def run(a, b, ev=None):
        n = b - a
        for k, _ in cols:
            dcols[k][:n].copy_(pin[k][a:b], non_blocking=True)
        if ev is not None:
            ev[0].record()
        p = sc.score(*(dcols[k][:n] for k, _ in cols))
        if ev is not None:
            ev[1].record()
        out_h[:n].copy_(p, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return n

    t_hist = time.perf_counter()
    for k in range(args.history_days):
        run(int(day_cuts[k]), int(day_cuts[k + 1]))
    sc.state.check()
    t_hist = time.perf_counter() - t_hist

    nb = len(bounds) - 1
    n_warm = min(args.warmup, max(nb - 1, 0))
    n_timed = nb - n_warm if args.batches <= 0 else min(args.batches, nb - n_warm)
    packed = None
    if wire is None and not args.column_copies:
        packed = [pack(int(bounds[k]), int(bounds[k + 1])) for k in range(n_warm + n_timed)]
        if graph:
            for n in sorted({b.numel() // 25 for b in packed}):
                sc.score_graph(*stage_views(n), out_host=out_h, replay=False)
    one = (lambda k, ev=None: run_packed(k, ev)) if packed is not None else \
        (lambda k, ev=None: run(int(bounds[k]), int(bounds[k + 1]), ev))
    for k in range(n_warm):
        if wire is not None:
            run_cdc(k)
        else:
            one(k)
    if world > 1:
        dist.barrier()
    lat, dev_ms, rows = [], [], 0
    for k in range(n_warm, n_warm + n_timed):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        t0 = time.perf_counter()
        rows += run_cdc(k, ev) if wire is not None else one(k, ev)
        lat.append((time.perf_counter() - t0) * 1e3)
        dev_ms.append(ev[0].elapsed_time(ev[1]))
    sc.state.check()
    lat, dev_ms = np.array(lat), np.array(dev_ms)
    total_rows = rows
    if world > 1:
        t = torch.tensor(np.stack([lat, dev_ms]), dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lat, dev_ms = t[0].cpu().numpy(), t[1].cpu().numpy()
        r = torch.tensor([rows], dtype=torch.int64, device=cdev)
        dist.all_reduce(r)
        total_rows = int(r.item())
    out = {
        "metric": "config 5: micro-batch latency, incremental window-state update + RF(100, d20) scoring",
        "value": round(float(np.percentile(lat, 50)), 3),
        "unit": "ms (p50 per micro-batch, host batch in -> probabilities on host)"
                + ("; batches as Debezium wire columns (decode + dedup + compact on the device)" if args.cdc else ""),
        "p99_ms": round(float(np.percentile(lat, 99)), 3),
        "max_ms": round(float(lat.max()), 3),
        "device_p50_ms": round(float(np.percentile(dev_ms, 50)), 3),
        "device_p99_ms": round(float(np.percentile(dev_ms, 99)), 3),
        "tx_per_s": round(total_rows / (lat.sum() * 1e-3), 1),
        "higher_is_better": False,
        "n_gpus": world,
        "batches": int(n_timed),
        "warmup": int(n_warm),
        "mean_batch_tx": round(total_rows / max(n_timed, 1), 1),
        "dtype": "f64",
        **({"rehearsal": "--rehearse-one-gpu: every rank on one GPU, host-staged gloo collectives; not a "
                         "measurement"} if args.rehearse_one_gpu else {}),
        "data": "synthetic: handbook-distribution generator on the GPU (fdx.synth.generate_device, seed 4321, draws keyed by the global customer id)",
        "config": {"workload": f"configs[4]: tail of configs[3] ({args.customers} customers / {args.terminals} "
                               f"terminals), {args.history_days} days of history in the state, then day "
                               f"{args.history_days} as micro-batches of {args.batch} tx",
                   "parallelism": f"customer-sharded x{world}, terminal owner = id % {world}",
                   "state_bytes_per_gpu": sc.state.memory_bytes,
                   "rings": [args.customer_ring, args.terminal_ring]},
        "setup_s": {"generate": round(t_gen, 1), "history_stream": round(t_hist, 1)},
        "launch": ("one HIP graph per batch (state update, row assembly, forest, status and probabilities "
                   "copies; device_p50 includes the probabilities' copy to the host)"
                   if packed is not None and graph else "kernels enqueued one by one"),
        "host_input": ("Debezium wire columns, one pinned buffer per column" if args.cdc else
                       "five pinned columns, one copy each" if packed is None else
                       "one pinned buffer per batch, the five columns back to back (one host-to-device copy)"),
    }
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
