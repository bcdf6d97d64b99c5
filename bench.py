"""Headline benchmark: transactions/s featurized + scored, and % of the HBM roofline.

A step = one pass of the hot path over one batch already resident in HBM:
  re-key by CUSTOMER_ID -> customer 1/7/30-day windows -> re-key by TERMINAL_ID ->
  terminal delayed-risk windows -> time flags + assemble the 15 input_features +
  StandardScaler -> RandomForest(100 trees, depth 20) predict_proba.
Workload (plan_workload):
  N = 1: BASELINE.json configs[1] -- 50k customers / 100k terminals / 183 days (~17.7M tx);
  N > 1: BASELINE.json configs[3] -- 1M customers / 2M terminals / 365 days (~700M tx) IN
         TOTAL, strong scaling: rank r owns the contiguous CUSTOMER_ID range
         [r * 1M / N, (r + 1) * 1M / N) and all its rows; the 2M terminals are one shared id
         space (owner = id % N) whatever N is.
Synthetic data from the handbook distributions generated on the GPU (fdx.synth.generate_device;
no host generation inside the GPU lease), scored with the config-3 model
(bench_assets/rf100_d20.npz, trained with sklearn on config-1 features).

N GPUs: one process per GPU.  Launched by torch.distributed.run (RANK / WORLD_SIZE set) or,
when `--gpus N > 1` is given without WORLD_SIZE, this script starts the N ranks itself
(child processes, before anything touches the GPU) and exits with their status.  The
terminal half runs after an RCCL all-to-all re-key (fdx.distributed).  Rank 0 prints one
JSON line.

Per-kernel roofline: every stage of a step is bracketed by HIP events on
the stream it runs on, inside the timed steps; the JSON line carries, per stage, the
§8(d) algorithmic bytes per transaction, the mean time, the achieved GB/s and its fraction
of the 8 TB/s HBM peak, plus the HBM traffic rocprofv3 measured for its kernels
(profiles/pmc_kernels.json) when that file covers them.
"""
import argparse
import json
import os
import subprocess
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
# (round 4 also printed a "measured random-read ceiling" from tools/lds_probe.hip's wall-clock rate
# of bank-conflicted reads; it is dropped: the walk's own counters -- the LDS array's busy share
# and the waves' s_waitcnt share, from profiles/pmc_kernels.json -- say how close it runs)

# SURVEY.md §8(d) algorithmic bytes per transaction (compact logical I/O, read once + write once)
ALG = {"K2": 30, "K1-cust": 58, "K1-term": 49, "K3": 90, "end-to-end": 107}
# what one step actually reads and writes per transaction, end to end: the raw columns in (ts 8,
# customer 4, terminal 4, amount 8, fraud 1 = 25 B), proba out (8 B), and -- with the featurized
# table emitted -- the 14 feature columns in §8(d)'s compact form (3 x int32 + 3 x f64 per half,
# 2 x u8 flags = 74 B; the fdx_feature_row record pads them to 80 B, counted at 74)
E2E_IN, E2E_PROBA, E2E_FEATURES = 25, 8, 74
# bench stages (marks of FraudPipeline.run_fused) -> §8(d) unit and the kernels they launch
# (substring of the rocprofv3 kernel name, dispatches per step; "chunks" = forest chunks)
STAGES = [
    ("rekey_customer", "K2", [("k_radix_hist<unsigned int, 8>", 2), ("k_radix_scatter<unsigned int, 8, 2>", 2)]),
    ("customer_layout", "K1-cust", [("k_interleave<true, true>", 1)]),
    ("customer_walk", "K1-cust", [("k_customer_walk", 1)]),
    ("rekey_terminal", "K2", [("k_radix_hist<unsigned int, 9>", 1), ("k_radix_scatter<unsigned int, 9, 1>", 1),
                              ("k_radix_scatter<unsigned int, 8, 1>", 1)]),  # 17-bit ids: a 9- and an 8-bit pass
    ("terminal_windows", "K1-term", [("k_terminal_short<3>", 1), ("k_terminal_g<false, 1024>", 1)]),
    ("assemble_rows", "K3", [("k_zfill_grouped_w3", 1)]),
    ("forest_traverse", "K3", [("k_forest_rank", "chunks")]),
]
# N > 1 (ShardedPipeline): the terminal half is the exchange on the side stream instead
EXCHANGE_STAGES = [
    ("exchange_splits", "xGMI", [("k_key_map", 1), ("k_radix_hist", 1), ("k_radix_scatter", 1)]),
    ("exchange_pack", "xGMI", [("k_exchange_pack", 1)]),
    ("exchange_rows", "xGMI", []),
    ("owner_windows", "K1-term", [("k_exchange_unpack", 1), ("k_radix_scatter<unsigned int, 9, 1>", 1),
                                  ("k_radix_scatter<unsigned int, 8, 1>", 1),
                                  ("k_terminal_g<true>", 1)]),
    ("exchange_back", "xGMI", []),
]
XGMI_LINK_GBS = 153.0  # per point-to-point xGMI link and direction (7 links per GPU)


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


def pmc_counters(name_part):
    """The committed SQ counters, per dispatch (profiles/pmc_kernels.json), of the busiest kernel
    whose name contains name_part (the most wave-cycles: e.g. the forest's chunk-loop
    instantiation, not the per-chunk one a small check batch runs), or {}."""
    p = os.path.join(ROOT, "profiles", "pmc_kernels.json")
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        d = json.load(f)
    hits = [v for k, v in d["kernels"].items() if name_part in k]
    return max(hits, key=lambda v: v.get("SQ_WAVE_CYCLES", 0.0)) if hits else {}


def pmc_table():
    """{kernel name: HBM bytes per dispatch} from the committed rocprofv3 PMC summary
    (FETCH_SIZE / WRITE_SIZE passes; correction as stated in that file), or {}."""
    p = os.path.join(ROOT, "profiles", "pmc_kernels.json")
    if not os.path.exists(p):
        return {}, None
    with open(p) as f:
        d = json.load(f)
    return {k: v["hbm_bytes_per_dispatch"] for k, v in d["kernels"].items() if "hbm_bytes_per_dispatch" in v}, \
        "profiles/pmc_kernels.json" + (f" (rocprofv3 run {d['source']})" if d.get("source") else "")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("auto", "configs1", "configs3"), default="auto",
                    help="auto: configs[1] per GPU at N = 1, configs[3] split over the ranks at N > 1")
    ap.add_argument("--customers", type=int, default=None, help="override: customers (per GPU for configs1, "
                                                                 "in total for configs3)")
    ap.add_argument("--terminals", type=int, default=None, help="override: terminals (as --customers)")
    ap.add_argument("--days", type=int, default=None)
    ap.add_argument("--model", default=os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-score-rows", type=int, default=200_000,
                    help="rows of the sklearn predict_proba sample in the CPU baseline")
    ap.add_argument("--forest-variant", type=int, default=-1,
                    help="traversal kernel shape (fdx_forest_set_variant; -1 = the library default)")
    ap.add_argument("--avg-mode", choices=("exact", "scan"), default="exact",
                    help="customer averages: pandas-exact recurrence (default) or float64 prefix sums (SURVEY §7.4)")
    ap.add_argument("--isolated-steps", type=int, default=5,
                    help="extra steps after the timed region with every stage on one stream (one more untimed "
                         "first): per-kernel times for the roofline table (median)")
    ap.add_argument("--sweep-variant", default="", help="comma list of forest variants to time (stderr)")
    ap.add_argument("--wide-records", action="store_true",
                    help="terminal count records in the 24-byte form (FraudPipeline(compact_records=False); "
                         "default: the 16-byte compact form)")
    ap.add_argument("--emit-features", choices=("slot", "input", "none"), default="slot",
                    help="the featurized table every step writes besides scoring: the 14 feature columns per "
                         "transaction in SURVEY.md §8(d)'s compact form + the row index, as columns by scoring slot "
                         "(default, coalesced: ops.FeatureTable) or as 80-byte records by input row (one random "
                         "write per row: ops.FeatureRecords); none: scores only")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="rehearsal of the N > 1 orchestration on a one-GPU box: every rank on cuda:0, a gloo "
                         "process group, the exchange's two collectives staged through host memory (RCCL needs a "
                         "GPU per rank); the line is marked \"rehearsal\" and its timing is not a measurement")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU (RCCL all-to-all) path even at 1 GPU (measures its overhead)")
    return ap.parse_args()


# BASELINE.json configs: [1] = 50k / 100k / 183 days on one GPU, [3] = 1M / 2M / 365 days on 8
WORKLOADS = {"configs1": (50_000, 100_000, 183), "configs3": (1_000_000, 2_000_000, 365)}


def plan_workload(world, rank, workload="auto", customers=None, terminals=None, days=None):
    """This rank's share of the bench workload.
    configs1 (weak scaling, the N = 1 default): every rank owns its own `customers` customers
      [rank * C, (rank + 1) * C) and the terminal id space grows to terminals * world;
    configs3 (strong scaling, the N > 1 default): `customers` customers IN TOTAL, rank r owns
      the contiguous range [r * C // world, (r + 1) * C // world); the terminal id space is
      `terminals` whatever the world size.
    -> dict(name, scaling, customer_base, n_customers_local, n_customers_total,
            n_terminals_total, days)"""
    name = workload if workload != "auto" else ("configs1" if world == 1 else "configs3")
    c0, t0, d0 = WORKLOADS[name]
    C = c0 if customers is None else int(customers)
    T = t0 if terminals is None else int(terminals)
    D = d0 if days is None else int(days)
    if name == "configs1":
        return {"name": name, "scaling": "weak", "customer_base": rank * C, "n_customers_local": C,
                "n_customers_total": C * world, "n_terminals_total": T * world, "days": D}
    lo, hi = rank * C // world, (rank + 1) * C // world
    return {"name": name, "scaling": "strong", "customer_base": lo, "n_customers_local": hi - lo,
            "n_customers_total": C, "n_terminals_total": T, "days": D}


SCALE_REF = os.path.join(ROOT, "profiles", "configs3_n1.json")


def scale_reference(wl):
    """The N = 1 measurement of the configs[3] table (profiles/configs3_n1.json: the JSON line of
    `bench.py --gpus 1 --workload configs3`), or why there is none."""
    ref = {"n_gpus": 1, "workload": "configs3", "source": os.path.relpath(SCALE_REF, ROOT)}
    if wl["name"] != "configs3":
        return dict(ref, value=None, note="this line is not the configs[3] table")
    try:
        with open(SCALE_REF) as f:
            line = json.load(f)
    except (OSError, ValueError):
        return dict(ref, value=None, note="no committed N = 1 line")
    same = line.get("config", {}).get("global_tx")
    ref.update(value=line.get("value"), ms_per_step=line.get("ms_per_step"), global_tx=same,
               error=line.get("error"))
    return ref


def median(v):
    v = sorted(v)
    m = len(v) // 2
    return v[m] if len(v) % 2 else 0.5 * (v[m - 1] + v[m])


# an isolated stage time (the stage alone on one stream) above this multiple of the same stage's
# in-step time (beside the other stream's stages) cannot be a kernel time: it has absorbed
# something else (an allocation, a cold pool) and the table falls back to the in-step time
ISOLATED_MAX_OVER_IN_STEP = 2.0


def stage_table(in_step, isolated, stages):
    """Per-stage timing rows.  in_step / isolated: {stage: [ms per step]}; stages: the
    (name, unit, kernels) list.  ms_in_step / ms_isolated are MEDIANS over the steps; `ms` (what
    the rooflines use) is the isolated time unless it exceeds ISOLATED_MAX_OVER_IN_STEP x the
    in-step time, in which case the isolated sample is rejected (kept as ms_isolated_rejected)."""
    table = []
    for name, unit, kernels in stages:
        if name not in in_step:
            continue
        row = {"stage": name, "unit": unit, "ms_in_step": round(median(in_step[name]), 4)}
        row["ms"] = row["ms_in_step"]
        if isolated and name in isolated:
            iso = round(median(isolated[name]), 4)
            if iso > ISOLATED_MAX_OVER_IN_STEP * row["ms_in_step"]:
                row["ms_isolated_rejected"] = iso
            else:
                row["ms_isolated"] = iso
                row["ms"] = iso
        row["kernels"] = [k for k, _ in kernels]
        table.append(row)
    return table


def spawn_ranks(n):
    """Start n ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), wait, return
    the worst exit status.  Runs before this process touches the GPU."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + sys.argv, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, abs(p.wait()))
    return rc


def stdout_to_stderr():
    """Route this process's fd 1 to stderr (RCCL prints a version banner on stdout when a
    communicator comes up) and return a file for the one JSON line on the real stdout."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def load_model(path):
    import numpy as np

    z = np.load(path)
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    return arrays, z["mean"], z["scale"], z["check_X"], z["check_proba"]


def host_info():
    """The GPU box's host CPUs as this process sees them."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0))
    try:
        import joblib

        jobs = int(joblib.cpu_count())  # respects cgroup CPU quotas (the box's CPU share)
    except Exception:  # noqa: BLE001
        jobs = usable
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": usable, "joblib_cpus": jobs}


def sklearn_forest(arrays, n_features=15):
    """A fitted sklearn RandomForestClassifier rebuilt from the saved node arrays (the bench
    model is stored as arrays, not a pickle): Tree.__setstate__ with sklearn's own node
    record layout.  Its predict_proba[:, 1] is checked against the saved sklearn output."""
    import numpy as np
    import sklearn.ensemble
    import sklearn.tree
    from sklearn.tree._tree import Tree

    off = arrays["node_offsets"]
    ests = []
    for t in range(len(off) - 1):
        lo, hi = int(off[t]), int(off[t + 1])
        n = hi - lo
        tree = Tree(n_features, np.array([2], dtype=np.intp), 1)
        dt = tree.__getstate__()["nodes"].dtype
        nodes = np.zeros(n, dtype=dt)
        nodes["left_child"] = arrays["left"][lo:hi]
        nodes["right_child"] = arrays["right"][lo:hi]
        leaf = nodes["left_child"] < 0
        nodes["feature"] = np.where(leaf, -2, arrays["feature"][lo:hi])
        nodes["threshold"] = np.where(leaf, -2.0, arrays["threshold"][lo:hi])
        nodes["n_node_samples"] = 1
        nodes["weighted_n_node_samples"] = 1.0
        if "missing_go_to_left" in dt.names:
            nodes["missing_go_to_left"] = arrays["missing_left"][lo:hi]
        v1 = arrays["value1"][lo:hi]
        values = np.stack([1.0 - v1, v1], axis=1).reshape(n, 1, 2)
        depth = np.zeros(n, np.int64)
        for i in range(n):
            if nodes["left_child"][i] >= 0:
                depth[nodes["left_child"][i]] = depth[nodes["right_child"][i]] = depth[i] + 1
        tree.__setstate__({"max_depth": int(depth.max()), "node_count": n, "nodes": nodes,
                           "values": np.ascontiguousarray(values)})
        est = sklearn.tree.DecisionTreeClassifier()
        est.tree_, est.n_outputs_, est.n_classes_, est.classes_ = tree, 1, 2, np.array([0, 1])
        est.n_features_in_, est.max_features_ = n_features, n_features
        ests.append(est)
    rf = sklearn.ensemble.RandomForestClassifier(n_estimators=len(ests))
    rf.estimators_, rf.n_outputs_, rf.n_classes_, rf.classes_ = ests, 1, 2, np.array([0, 1])
    rf.n_features_in_ = n_features
    return rf


def cpu_baseline(data, arrays, mean, scale, check_X, check_proba, score_rows):
    """The reference CPU path on this host, on bounded samples of the same workload:
      featurization -- the C port of the reference's pandas arithmetic (oracle/fdx_oracle.c,
        1 thread; FASTER than pandas' per-group apply, so a conservative baseline) over the
        WHOLE table (customer and terminal windows see every row);
      scoring -- scikit-learn itself (the reference's library): StandardScaler.transform +
        RandomForest predict_proba of the bench model, n_jobs=1 and n_jobs=-1, whole batch and
        in 10k-row Spark-UDF-shaped batches (fraud_detection.py:183-195, Arrow maxRecordsPerBatch).
    value = 1 / (featurize s/tx + scoring s/tx at n_jobs=-1 whole batch)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    import sklearn.preprocessing

    info = host_info()
    n = len(data["ts"])
    t0 = time.perf_counter()
    f = oracle.featurize_arrays(data["ts"], data["customer"], data["terminal"], data["amount"], data["fraud"])
    t_feat = time.perf_counter() - t0
    names = ["TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + oracle.CUSTOMER_COLS + oracle.TERMINAL_COLS
    m = min(score_rows, n)
    X = np.column_stack([data["amount"][:m]] + [f[k][:m] for k in names])
    rf = sklearn_forest(arrays)
    sc = sklearn.preprocessing.StandardScaler()
    sc.mean_, sc.scale_, sc.var_ = mean, scale, scale * scale
    sc.n_features_in_, sc.n_samples_seen_ = 15, 1
    rf.set_params(n_jobs=1)
    if not np.array_equal(rf.predict_proba(sc.transform(check_X))[:, 1], check_proba):
        raise SystemExit("rebuilt sklearn forest disagrees with the saved sklearn output")
    res = {}
    for jobs in (1, -1):
        rf.set_params(n_jobs=jobs)
        t0 = time.perf_counter()
        rf.predict_proba(sc.transform(X))
        res[f"whole_n_jobs{jobs}"] = m / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        for a in range(0, m, 10_000):
            rf.predict_proba(sc.transform(X[a:a + 10_000]))
        res[f"udf10k_n_jobs{jobs}"] = m / (time.perf_counter() - t0)
    feat_rate = n / t_feat
    value = 1.0 / (1.0 / feat_rate + 1.0 / res["whole_n_jobs-1"])
    return {"value": round(value, 1), "unit": "tx/s", "cores": info["joblib_cpus"], "kind": "port",
            "sample": f"featurize: C port of the pandas windows (1 thread) over all {n} tx of rank 0's batch, "
                      f"{t_feat:.1f} s; score: sklearn StandardScaler + RandomForest(100, d20) predict_proba on "
                      f"the first {m} rows (n_jobs=-1 = {info['joblib_cpus']} threads)",
            "featurize_tx_per_s": round(feat_rate, 1),
            "sklearn_rows_per_s": {k: round(v, 1) for k, v in res.items()},
            "host": info}


def rehearse_host_collectives():
    """--rehearse-one-gpu: the exchange's two collectives (fdx.distributed.all_to_all_split_pairs
    and alltoallv, module-level for this) copy their device buffers through host memory and run
    the same gloo all-to-all / batched point-to-point there; everything else is the product path
    (as tests/test_gpu_aa_sharded_world2.py does)."""
    import torch
    import torch.distributed as dist

    from fdx import distributed as D

    staged_v = D.alltoallv

    def pairs_host(out, inp, group=None):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), group=group)
        out.copy_(h)
        return out

    def alltoallv_host(out, inp, out_splits, in_splits, group=None):
        h = torch.empty(out.shape, dtype=out.dtype)
        staged_v(h, inp.cpu(), out_splits, in_splits, group)
        out.copy_(h)
        return out

    D.all_to_all_split_pairs, D.alltoallv = pairs_host, alltoallv_host


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    json_out = stdout_to_stderr()
    _STATE["json_out"] = json_out
    import numpy as np
    import torch
    import torch.distributed as dist

    from fdx import _lib, ops, synth
    from fdx.pipeline import FraudPipeline

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    cdev = torch.device("cpu") if args.rehearse_one_gpu else dev  # bench's own reductions
    if world > 1 and args.rehearse_one_gpu:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus, f"world {dist.get_world_size()} != --gpus {args.gpus}"
        rehearse_host_collectives()
    elif world > 1:
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus, f"world {dist.get_world_size()} != --gpus {args.gpus}"
    elif args.sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)

    wl = plan_workload(world, rank, args.workload, args.customers, args.terminals, args.days)
    base, n_cl, n_terms = wl["customer_base"], wl["n_customers_local"], wl["n_terminals_total"]
    t_gen = time.perf_counter()
    # generated on the GPU (HIP Philox generator, csrc/fdx_synth.hip): the handbook
    # distributions of fdx.synth.generate, pinned by tests/test_gpu_synth.py; inputs resident
    # one population for every N: rank r draws the rows of ITS customers of the same population
    # (draws keyed by the global customer id, tests/test_gpu_synth.py), so the union over the
    # ranks is the same table at N = 1, 2, 4, 8
    g = synth.generate_device(n_cl, n_terms, wl["days"], seed=1234, customer_offset=base,
                              n_customers_total=wl["n_customers_total"], device=dev)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen
    n_local = g["ts"].numel()
    _STATE.update(tx_per_gpu=n_local, workload=wl["name"], n_customers_local=n_cl, days=wl["days"])
    arrays, mean, scale, check_X, check_proba = load_model(args.model)
    forest = ops.Forest(arrays, 15, mean, scale)
    default_variant = forest.variant
    if args.forest_variant >= 0:
        forest.set_variant(args.forest_variant)
    T = lambda a, d: torch.from_numpy(np.ascontiguousarray(a)).to(dev, d)  # noqa: E731
    # sanity: the GPU forest reproduces sklearn on the held-out sample saved with the model
    got = forest.predict(T(check_X, torch.float64)).cpu().numpy()
    if not np.array_equal(got, check_proba):
        raise SystemExit("forest parity check against sklearn failed")

    ts, cust, term, amt, fr = g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"]
    pipe = FraudPipeline(forest=forest, avg_mode=args.avg_mode, compact_records=not args.wide_records)
    ws = ops.workspace(forest.workspace_size(n_local * 11 // 10), dev)  # scoring slots incl. layout padding
    proba = torch.empty(n_local, dtype=torch.float64, device=dev)
    emit = args.emit_features != "none"
    # the featurized table: one record per scoring slot (incl. the layout's padding) or per row
    rows_out = None if not emit else (ops.FeatureTable(n_local * 11 // 10, dev) if args.emit_features == "slot"
                                      else ops.FeatureRecords(n_local, dev))
    marks_all = []   # per timed step: {stage: (start event, end event)}
    trav = []        # per timed step: (start, end) of the forest traversal
    shard_stats = {}  # the exchange's split sizes / bytes per peer (N > 1)

    def make_mark(record):
        """mark(stage, stream): a HIP event on the stage's stream, paired with the previous
        event on that stream ("start" opens a stream); marks[stage] = (start, end)."""
        marks, last = {}, {}

        def mark(name, st):
            if record:
                e = torch.cuda.Event(enable_timing=True)
                e.record(st)
                if name == "start":
                    marks.setdefault("_starts", []).append(e)
                else:
                    marks[name] = (last[id(st)], e)
                last[id(st)] = e
        return mark, marks

    if world > 1 or args.sharded:
        from fdx.distributed import ShardedPipeline

        sp = ShardedPipeline(pipe, world, rank, n_terms, customer_base=base, n_customers_local=n_cl)

        def step(record):
            mark, marks = make_mark(record)
            sp.run(ts, cust, term, amt, fr, proba, ws, mark=mark, stats=shard_stats, rows_out=rows_out)
            if record:
                marks_all.append(marks)
                trav.append(marks["forest_traverse"])
    else:
        lcust = cust  # rank 0 of a 1-GPU run: base 0

        def step(record, overlap=True, into=None):
            mark, marks = make_mark(record)
            pipe.run_fused(ts, lcust, term, amt, fr, n_cl, n_terms, proba, ws, mark=mark, overlap=overlap,
                           rows_out=rows_out)
            if record and into is not None:
                into.append(marks)
            elif record:
                marks_all.append(marks)
                trav.append(marks["forest_traverse"])

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    mem0 = torch.cuda.memory_stats(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    mem1 = torch.cuda.memory_stats(dev)
    # the caching allocator inside the timed steps: device allocations / frees / OOM retries there
    # mean the steps paid hipMalloc / hipFree (each hipFree synchronises the device)
    allocator = {k: int(mem1.get(k, 0) - mem0.get(k, 0)) for k in ("num_device_alloc", "num_device_free",
                                                                  "num_alloc_retries")}
    allocator.update(peak_reserved_GB=round(mem1.get("reserved_bytes.all.peak", 0) / 1e9, 2),
                     peak_allocated_GB=round(mem1.get("allocated_bytes.all.peak", 0) / 1e9, 2),
                     conf=os.environ.get("PYTORCH_HIP_ALLOC_CONF") or os.environ.get("PYTORCH_CUDA_ALLOC_CONF"))
    if world > 1:
        t = torch.tensor([dt, float(n_local)], dtype=torch.float64, device=cdev)
        dtm = t[:1].clone()
        dist.all_reduce(dtm, op=dist.ReduceOp.MAX)
        tot = t[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dt, n_total = float(dtm.item()), int(tot.item())
    else:
        n_total = n_local

    iso_all = []  # per-kernel times: every stage alone on the GPU (after the timed region)
    if marks_all and args.isolated_steps > 0 and not (world > 1 or args.sharded):
        # one untimed step in this mode first: its buffers come from the caller stream's pool,
        # which the overlapped steps (on the pipeline's own streams) never warmed -- the first
        # such step absorbs that pool's allocations (BENCH_r03: 5.65 / 7.57 / 7.92 ms "isolated"
        # stages of one cold step in a mean of 3)
        step(False, overlap=False)
        torch.cuda.synchronize()
        for _ in range(args.isolated_steps):
            step(True, overlap=False, into=iso_all)
        torch.cuda.synchronize()
    trav_ms = sum(a.elapsed_time(b) for a, b in trav) / max(len(trav), 1)
    launches = forest.traverse_launches(n_local)
    fvar = forest.variant
    # §8(d): K3 = 90 B per transaction (15 features in, proba out), over the traversal time
    achieved = ALG["K3"] * n_local / (trav_ms * 1e-3) / 1e9
    pmc, pmc_src = pmc_table()

    def pmc_bytes(kernels):
        tot, seen = 0.0, True
        for sub, cnt in kernels:
            hits = [v for k, v in pmc.items() if sub in k]
            if not hits:
                seen = False
                continue
            tot += max(hits) * (launches if cnt == "chunks" else cnt)
        return tot if seen and pmc else None

    fk = [v for k, v in pmc.items() if "k_forest_rank" in k]
    out = {
        "metric": METRIC,
        "value": round(n_total * args.steps / dt, 1),
        "unit": "tx/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "setup_s": {"generate_on_gpu": round(t_gen, 2)},
        "allocator_in_timed_steps": allocator,
        **({"rehearsal": "--rehearse-one-gpu: every rank on one GPU, host-staged gloo collectives; not a "
                         "measurement"} if args.rehearse_one_gpu else {}),
        "data": "synthetic: handbook-distribution generator on the GPU (fdx.synth.generate_device, seed 1234, "
                "draws keyed by the global customer id: each rank's rows are the population's rows of its customer "
                "range, the union is the same table at every N), resident in HBM",
        "config": {"workload": (f"configs[1]: {n_cl} customers / {n_terms // world} terminals / {wl['days']} days "
                                f"per GPU" if wl["name"] == "configs1" else
                                f"configs[3]: {wl['n_customers_total']} customers / {n_terms} terminals / "
                                f"{wl['days']} days in total, contiguous customer ranges over {world} GPU(s)")
                               + ", featurize + RF(100 trees, depth 20) predict_proba",
                   "customer_range": [base, base + n_cl],
                   "tx_per_gpu": n_local, "global_tx": n_total,
                   "parallelism": f"customer-sharded x{world}" + (" (RCCL all-to-all re-key)" if world > 1 else ""),
                   "model": "bench_assets/rf100_d20.npz (sklearn RandomForest, config-1 features)",
                   "customer_averages": args.avg_mode,
                   "features_emitted": args.emit_features},
        "roofline": {"kernel": "k_forest_rank", "bound": "hbm", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": round(max(fk)) if fk else None, "traffic_unit": "HBM bytes per launch (PMC)",
                     "algorithmic_bytes_per_launch": round(ALG["K3"] * n_local / launches),
                     "algorithmic_bytes_per_tx": ALG["K3"], "avg_launch_ms": round(trav_ms / launches, 4),
                     "launches_per_step": launches, "traverse_ms": round(trav_ms, 3), "forest_variant": fvar,
                     "traffic_source": pmc_src},
    }
    steps_max = walk_steps_per_row(arrays)
    ach_steps = steps_max * n_local / (trav_ms * 1e-3)
    out["roofline_lds"] = {"kernel": "k_forest_rank", "bound": "lds", "unit": "node steps/s",
                           "achieved": float(f"{ach_steps:.4g}"), "peak": float(f"{LDS_PEAK_STEPS:.4g}"),
                           "frac": round(ach_steps / LDS_PEAK_STEPS, 4), "node_steps_per_row_max": steps_max,
                           "note": "peak = the LDS array's conflict-free rate: 2 ds_read_b32 per step at 2 LDS "
                                   "cycles each (MI355X_MICROARCH.md §LDS); steps = sum of tree depths (upper "
                                   "bound: wave-wide early exit), so frac is an upper bound"}
    sq = pmc_counters("k_forest_rank")
    if sq.get("SQ_LDS_IDX_ACTIVE") and sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_WAVE_CYCLES"):
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles: per-CU cycles = it / 8; SQ_LDS_IDX_ACTIVE
        # sums every CU's LDS-array cycles; the SQ_WAIT / WAVE counters share one unit
        cu_cycles = sq["GRBM_GUI_ACTIVE"] / 8
        out["roofline_lds"]["pmc"] = {
            "lds_array_busy_share": round(sq["SQ_LDS_IDX_ACTIVE"] / 256 / cu_cycles, 3),
            "lds_bank_conflict_share": round(sq.get("SQ_LDS_BANK_CONFLICT", 0) / sq["SQ_LDS_IDX_ACTIVE"], 3),
            "wave_waitcnt_share": round(sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"], 3),
            "wave_issue_stall_share": round(sq.get("SQ_WAIT_INST_ANY", 0) / sq["SQ_WAVE_CYCLES"], 3),
            "valu_busy_share": round(sq.get("SQ_INSTS_VALU", 0) / 1024 * 2 / cu_cycles, 3),
            "source": "profiles/pmc_kernels.json (per dispatch; VALU at 2 cycles per wave64 instruction "
                      "on SIMD-32, 1,024 SIMDs)"}
    if marks_all:
        ms_of = lambda steps: {name: [mk[name][0].elapsed_time(mk[name][1]) for mk in steps]  # noqa: E731
                               for name in steps[0] if not name.startswith("_")}
        table = stage_table(ms_of(marks_all), ms_of(iso_all) if iso_all else None, STAGES + EXCHANGE_STAGES)
        for row in table:
            row["pmc_bytes"] = pmc_bytes(next(k for n_, _, k in STAGES + EXCHANGE_STAGES if n_ == row["stage"]))
        # §8(d) units: K1-cust = layout + walk, K3 = assemble + traverse
        units = {}
        for row in table:
            if row["unit"] == "xGMI":
                continue
            u = units.setdefault(row["unit"] + ("" if row["unit"] != "K2" else ":" + row["stage"]),
                                 {"ms": 0.0, "stages": [], "pmc": 0.0, "pmc_ok": True})
            u["ms"] += row["ms"]
            u["stages"].append(row["stage"])
            if row["pmc_bytes"] is None:
                u["pmc_ok"] = False
            else:
                u["pmc"] += row["pmc_bytes"]
        krows = []
        for key, u in units.items():
            unit = key.split(":")[0]
            alg = ALG[unit] * n_local
            gbs = alg / (u["ms"] * 1e-3) / 1e9
            krows.append({"unit": unit, "stages": u["stages"], "alg_bytes_per_tx": ALG[unit],
                          "ms": round(u["ms"], 4), "achieved_GBs": round(gbs, 1),
                          "frac": round(gbs / HBM_PEAK_GBS, 4),
                          "pmc_traffic_bytes": round(u["pmc"]) if u["pmc_ok"] and pmc else None,
                          "traffic_over_alg": round(u["pmc"] / alg, 2) if u["pmc_ok"] and pmc else None})
        step_ms = sum(r["ms_in_step"] for r in table)
        e2e_b = E2E_IN + E2E_PROBA + (E2E_FEATURES if emit else 0)
        e2e = e2e_b * n_local / (dt / args.steps) / 1e9
        out["kernels"] = {"per_stage": table, "per_unit": krows, "stage_sum_ms": round(step_ms, 3),
                          "streams": "rekey_terminal + terminal_windows run on a side stream, concurrently with the "
                                     "customer stages, so stage_sum_ms (of ms_in_step) exceeds ms_per_step by the "
                                     "overlap; ms = ms_isolated: the same stages in extra steps with every stage on "
                                     "one stream (no concurrent kernel; median of --isolated-steps after one untimed step in "
                                     "that mode), the per-kernel durations the rooflines use; an isolated time "
                                     f"above {ISOLATED_MAX_OVER_IN_STEP}x the in-step time is rejected "
                                     "(ms_isolated_rejected) and ms falls back to ms_in_step",
                          "end_to_end": {"alg_bytes_per_tx": e2e_b, "achieved_GBs": round(e2e, 1),
                                         "time": "ms_per_step", "features_emitted": args.emit_features,
                                         "bytes": f"raw columns in {E2E_IN} + proba out {E2E_PROBA}"
                                                  + (f" + feature columns out {E2E_FEATURES} (the 14 "
                                                     f"columns in §8(d)'s compact logical form; the table as "
                                                     f"written by {args.emit_features} adds the row index and "
                                                     f"padding: 78 B per slot / 80 B per record)" if emit
                                                     else " (featurized table not written: --emit-features none)")
                                                  + f"; SURVEY.md §8(d)'s fused ideal is {ALG['end-to-end']}",
                                         "frac": round(e2e / HBM_PEAK_GBS, 4)},
                          "note": "ms_in_step = HIP events around each stage on its stream, median over the timed steps; "
                                  "alg bytes = SURVEY.md §8(d) per tx x tx; pmc = rocprofv3 FETCH/WRITE per "
                                  "dispatch x dispatches (profiles/pmc_kernels.json)"}
    if marks_all and (world > 1 or args.sharded):
        # the exchange against the xGMI link roofline, and how much of it the customer half hides
        def span(mk, a, b):  # ms from event a to event b
            return a.elapsed_time(b)

        ex_ms, link_ms, hidden_ms = [], [], []
        for mk in marks_all:
            t0m = mk["_starts"][0]                      # main stream start
            ex_a, ex_b = mk["exchange_splits"][0], mk["exchange_back"][1]
            cu_b = mk["customer_walk"][1]
            a, b = span(mk, t0m, ex_a), span(mk, t0m, ex_b)
            c = span(mk, t0m, cu_b)
            ex_ms.append(b - a)
            hidden_ms.append(max(0.0, min(b, c) - max(a, 0.0)))
            link_ms.append(span(mk, *mk["exchange_rows"]) + span(mk, *mk["exchange_back"]))
        mean = lambda v: sum(v) / len(v)  # noqa: E731
        loc = torch.tensor([float(n_local), float(shard_stats.get("bytes_to_peers", 0)), mean(ex_ms), mean(link_ms),
                            mean(hidden_ms)], dtype=torch.float64, device=cdev)
        if world > 1:
            allr = [torch.empty_like(loc) for _ in range(world)]
            dist.all_gather(allr, loc)
            allr = torch.stack(allr).cpu().numpy()
        else:
            allr = loc.cpu().numpy()[None, :]
        peers = max(world - 1, 1)
        link_peak = min(peers, 7) * XGMI_LINK_GBS
        per_rank = []
        for r_ in range(world):
            n_r, b_r, e_r, l_r, h_r = allr[r_]
            per_rank.append({"rank": r_, "tx": int(n_r), "bytes_to_peers": int(b_r), "exchange_ms": round(e_r, 4),
                             "link_ms": round(l_r, 4),
                             "achieved_egress_GBs": round(b_r / (l_r * 1e-3) / 1e9, 1) if l_r > 0 else None,
                             "hidden_share": round(h_r / e_r, 3) if e_r > 0 else None})
        me = per_rank[rank]
        out["exchange"] = {
            "world": world, "per_rank": per_rank,
            "send_rows_per_peer": shard_stats.get("send_rows"), "recv_rows_per_peer": shard_stats.get("recv_rows"),
            "bytes_per_row": {"rows": shard_stats.get("row_bytes"), "reply": shard_stats.get("reply_bytes")},
            "link_roofline": {"bound": "xgmi", "peers": world - 1, "peak_GBs": link_peak,
                              "achieved_GBs": me["achieved_egress_GBs"],
                              "frac": round(me["achieved_egress_GBs"] / link_peak, 4)
                              if me["achieved_egress_GBs"] and world > 1 else None},
            "note": "exchange_ms = side-stream span from the owner-key re-key to the reply all-to-all; link_ms = "
                    "the two all-to-all phases (rows 16 B/row out, count records 24 B/row back); achieved = bytes "
                    "this rank sends to its peers / link_ms against min(world-1, 7) x 153 GB/s; hidden_share = "
                    "part of exchange_ms that overlaps the customer half (main-stream start to customer_walk end)"}
    if world > 1 or wl["name"] == "configs3":
        # the 1 -> N curve: configs[3] is strong scaling (the same 1M-customer table at every N), so
        # every N > 1 line names the N = 1 run of that same table it scales against (a committed
        # bench line: python bench.py --gpus 1 --workload configs3)
        out["scales_against"] = scale_reference(wl)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        data = {k: g[k].cpu().numpy() for k in ("ts", "customer", "terminal", "amount", "fraud")}
        out["cpu_baseline"] = cpu_baseline(data, arrays, mean, scale, check_X, check_proba, args.cpu_score_rows)
    if args.sweep_variant and rank == 0 and world == 1 and not args.sharded:
        # each variant: one full untimed pipeline pass (the prepared row format depends on
        # the layout), bit-equality of proba against the default, one untimed and 5 timed
        # traversals; the whole list twice (the first variant timed after the bench loop read
        # ~0.6 ms slow), min of the two rounds reported
        res = {}
        ref = proba.clone()
        vlist = [int(x) for x in args.sweep_variant.split(",")]
        for rnd in range(2):
            for v in vlist:
                forest.set_variant(v)
                pv = torch.empty_like(proba)
                try:
                    pipe.run_fused(ts, cust, term, amt, fr, n_cl, n_terms, pv, ws)
                except _lib.FdxError as e:  # e.g. a 32-slot v2 variant: the fused rows are v1-format only
                    res[v] = {"skipped": str(e)}
                    continue
                same = bool(torch.equal(pv, ref))
                wsv, n_rows = pipe._forest_ws(pipe.last_slots, ws, dev), pipe.last_slots
                buf = torch.empty(n_rows, dtype=torch.float64, device=dev)
                ops.forest_traverse(forest, n_rows, wsv, buf)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(5):
                    ops.forest_traverse(forest, n_rows, wsv, buf)
                b.record()
                torch.cuda.synchronize()
                ms = round(a.elapsed_time(b) / 5, 3)
                r_ = res.setdefault(v, {"ms_rounds": [], "chunks": forest.n_chunks, "bit_equal": True})
                r_["ms_rounds"].append(ms)
                r_["ms"] = min(r_["ms_rounds"])
                r_["bit_equal"] = r_["bit_equal"] and same
        forest.set_variant(args.forest_variant if args.forest_variant >= 0 else default_variant)
        print(json.dumps({"variant_sweep_traverse": res}), file=sys.stderr)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1 or args.sharded:
        dist.destroy_process_group()


def main_or_report_oom():
    """main(); a run whose working set does not fit HBM (e.g. --gpus 1 --workload configs3: the
    whole 1M-customer / 365-day table on one GPU) prints one JSON line with the error and the
    byte counts instead of a traceback"""
    import torch

    try:
        main()
    except torch.cuda.OutOfMemoryError as e:
        free, total = torch.cuda.mem_get_info()
        line = {"metric": METRIC, "value": None, "unit": "tx/s", "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                "error": "out of HBM: " + str(e).splitlines()[0][:400], "hbm_bytes_free": free,
                "hbm_bytes_total": total, "hbm_bytes_allocated_by_torch": torch.cuda.memory_allocated(),
                **{k: v for k, v in _STATE.items() if k != "json_out"}}
        print(json.dumps(line), file=_STATE.get("json_out") or sys.stdout, flush=True)
        sys.exit(3)


_STATE = {}

if __name__ == "__main__":
    main_or_report_oom()
