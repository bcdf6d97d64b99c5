"""BASELINE.json configs at full size, on the GPU, through the C ABI.

configs[1]  50k customers / 100k terminals / 183 days (~17.7M tx): the bench's fused scoring
            path (FraudPipeline.run_fused) must give, on EVERY row, the probability of the
            float64 path (featurize -> X -> Forest.predict), and the features of >= 100 sampled
            customers and terminals (all their rows) must equal the C oracle bit for bit.
configs[2]  RandomForest(100 trees, depth 20) predict_proba: the bench model's 4,096 held-out
            rows against sklearn's saved output, then 140M rows resampled from them (past one
            forest row range); the deployed model likewise at 20M rows.
multi-rank  the exchange kernels (pack / unpack / owner records / reply) with world = 4 and 8
            record formats, the all-to-all simulated on the host: every rank's features must
            equal the single-GPU featurize of the union (the gloo test swaps these kernels for
            numpy stand-ins; here the HIP kernels run).
"""
import os

import numpy as np
import pytest
import torch

import oracle
from fdx import _lib, ops, synth
from fdx.pipeline import FraudPipeline
from table_check import assert_same_features, table_as_X

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUST_COLS, TERM_COLS = oracle.CUSTOMER_COLS, oracle.TERMINAL_COLS


def T(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)


def _model():
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    return arrays, z


def _check_sampled_segments(d, X, n_sample=128, seed=0):
    """Customer features of n_sample customers and terminal features of n_sample terminals,
    all their rows, against the oracle run on exactly those rows."""
    rng = np.random.default_rng(seed)
    cust = rng.choice(np.unique(d["customer"]), n_sample, replace=False)
    m = np.isin(d["customer"], cust)
    f = oracle.featurize_arrays(d["ts"][m], d["customer"][m], d["terminal"][m], d["amount"][m], d["fraud"][m])
    got = X[m]
    np.testing.assert_array_equal(got[:, 1], f["TX_DURING_WEEKEND"])
    np.testing.assert_array_equal(got[:, 2], f["TX_DURING_NIGHT"])
    for j, c in enumerate(CUST_COLS):
        np.testing.assert_array_equal(got[:, 3 + j], f[c], err_msg=c)
    term = rng.choice(np.unique(d["terminal"]), n_sample, replace=False)
    m = np.isin(d["terminal"], term)
    f = oracle.featurize_arrays(d["ts"][m], d["customer"][m], d["terminal"][m], d["amount"][m], d["fraud"][m])
    got = X[m]
    for j, c in enumerate(TERM_COLS):
        np.testing.assert_array_equal(got[:, 9 + j], f[c], err_msg=c)
    return int(m.sum())


def test_config2_full_size_fused_path_every_row(dev):
    arrays, z = _model()
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    d = synth.generate(50_000, 100_000, 183, seed=1234)
    n = len(d["ts"])
    assert n > 17_000_000
    args = (T(d["ts"], torch.int64, dev), T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(d["amount"], torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    pipe = FraudPipeline(forest=forest)
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    rows = ops.FeatureTable(n * 11 // 10, dev)  # the bench step's own featurized table
    rows.buf.fill_(0xAB)
    pipe.run_fused(*args, 50_000, 100_000, proba, ws, rows_out=rows)
    fused = proba.cpu().numpy()
    m_slots = pipe.last_slots
    feats = pipe.featurize(*args, 50_000, 100_000)
    p64 = pipe.score(feats.X).cpu().numpy()
    np.testing.assert_array_equal(fused, p64)
    X = feats.X.cpu().numpy()
    # every feature of every row of the fused path's table (interleave + walk + assembly) equals
    # the float64 path's X, itself checked against the oracle on sampled segments below
    assert_same_features(table_as_X(rows, m_slots, d["amount"]), X, "config 2 fused table")
    del rows
    np.testing.assert_array_equal(X[:, 0], d["amount"])
    rows = _check_sampled_segments(d, X)
    assert rows > 10_000
    # the sampled rows' probabilities against the oracle forest on the oracle's features
    sel = np.random.default_rng(1).choice(n, 20_000, replace=False)
    np.testing.assert_array_equal(p64[sel], oracle.forest_predict(X[sel], arrays, z["mean"], z["scale"]))


def test_fused_path_past_one_forest_row_range(dev):
    """A fused step whose scoring slots exceed one forest row range (134,216,704 slots: the walk's
    32-bit offsets; a configs[3] rank at N = 2 or 4 holds 177M-354M transactions): the traversal
    runs range by range with proba scattered through the layout's irow, and every row's proba
    equals the float64 path's (featurize + score) on the same data."""
    arrays, z = _model()
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    g = synth.generate_device(400_000, 800_000, 183, seed=4242, device=dev)
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"])
    n = args[0].numel()
    pipe = FraudPipeline(forest=forest)
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 400_000, 800_000, proba)
    assert pipe.last_slots > 134_216_704
    assert forest.traverse_launches(pipe.last_slots) == 2
    p64 = pipe.score(pipe.featurize(*args, 400_000, 800_000).X)
    assert torch.equal(proba, p64)


def _resampled(n, n_src, seed, dev):
    """n row indices into n_src rows, drawn on the device from a fixed seed"""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return torch.randint(0, n_src, (n,), generator=g, device=dev, dtype=torch.int64)


def test_config3_rf100_d20_bench_model(dev):
    """configs[2]: RF(100, depth 20) predict_proba over 100M+ HBM-resident rows -- 140M rows
    resampled from the bench model's 4,096 held-out rows, so sklearn's saved output of each
    source row is the expectation of every copy.  140M is past one forest row range
    (134,216,704 rows: the walk's 32-bit offsets into 32-B rank rows), so the traversal runs two
    ranges and every row of the second is checked too."""
    arrays, z = _model()
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    cx, cp = z["check_X"], z["check_proba"]
    np.testing.assert_array_equal(forest.predict(T(cx, torch.float64, dev)).cpu().numpy(), cp)
    n = 140_000_000
    idx = _resampled(n, len(cx), 7, dev)
    Xd = T(cx, torch.float64, dev)[idx]
    ws = ops.workspace(forest.workspace_size(n), dev)
    assert forest.traverse_launches(n) == 2  # two row ranges, one chunk-loop launch each
    got = forest.predict(Xd, ws=ws)
    del Xd, ws
    want = T(cp, torch.float64, dev)[idx]
    bad = int((got != want).sum())
    assert bad == 0, f"{bad} of {n} rows differ from sklearn"
    assert torch.equal(got[134_216_704:], want[134_216_704:])


def test_fused_path_rejects_ids_out_of_range(dev):
    arrays, z = _model()
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    d = synth.generate(300, 500, 20, seed=4)
    n = len(d["ts"])
    cust = d["customer"].copy()
    cust[n // 2] = 300                      # one id past n_customers
    args = (T(d["ts"], torch.int64, dev), T(cust, torch.int32, dev), T(d["terminal"], torch.int32, dev),
            T(d["amount"], torch.float64, dev), T(d["fraud"], torch.uint8, dev))
    pipe = FraudPipeline(forest=forest)
    proba = torch.empty(n, dtype=torch.float64, device=dev)
    with pytest.raises(_lib.FdxError, match="customer ids"):
        pipe.run_fused(*args, 300, 500, proba)
    # a negative terminal id (the terminal re-key's count, read through the side stream)
    term = d["terminal"].copy()
    term[n // 3] = -4
    args = args[:1] + (T(d["customer"], torch.int32, dev), T(term, torch.int32, dev)) + args[3:]
    with pytest.raises(_lib.FdxError, match="terminal ids"):
        pipe.run_fused(*args, 300, 500, proba)
    # ids past 2^key_bits (they sort among the in-range keys by their low bits, so the grouping
    # is out of key order): still rejected, and no kernel reads outside its buffers meanwhile
    for bad_id in (512 + 5, (1 << 30) + 7):  # low 9 bits: 5 and 7
        cust = d["customer"].copy()
        cust[n // 4 :: 97] = bad_id
        args = args[:1] + (T(cust, torch.int32, dev), T(d["terminal"], torch.int32, dev)) + args[3:]
        with pytest.raises(_lib.FdxError, match="customer ids"):
            pipe.run_fused(*args, 300, 500, proba)
    # in range again: the same pipeline scores (nothing left over from the failed calls)
    args = args[:1] + (T(d["customer"], torch.int32, dev), T(d["terminal"], torch.int32, dev)) + args[3:]
    pipe.run_fused(*args, 300, 500, proba)
    torch.cuda.synchronize()


# ----------------------------------------------------------------- multi-rank dataflow
@pytest.mark.parametrize("world", [4, 8])
def test_exchange_kernels_world_gt1_host_simulated_all_to_all(dev, world):
    """Ranks r = 0..world-1 own customers [r*C, (r+1)*C); every step of fdx.distributed's
    exchange runs its HIP kernel; only the two all-to-alls are done on the host."""
    from fdx.distributed import GpuKernels as K

    C, n_terms = 150, 400
    shards = [synth.generate(C, n_terms, 70, r=25, seed=40 + r, customer_offset=C * r) for r in range(world)]
    for r, s in enumerate(shards):
        s["gid"] = s["tid"] + (r << 32)
    whole = {k: np.concatenate([s[k] for s in shards])
             for k in ("ts", "customer", "terminal", "amount", "fraud", "gid")}
    o = np.argsort(whole["ts"], kind="stable")
    whole = {k: v[o] for k, v in whole.items()}
    pipe = FraudPipeline()
    ref = pipe.featurize(*(T(whole[k], dt, dev) for k, dt in (("ts", torch.int64), ("customer", torch.int32),
                                                             ("terminal", torch.int32), ("amount", torch.float64),
                                                             ("fraud", torch.uint8))),
                         C * world, n_terms).X.cpu().numpy()
    ref_row = {int(g): i for i, g in enumerate(whole["gid"])}
    # phase 1 on every rank: owner keys, re-key by owner, pack
    sent = []
    for r, s in enumerate(shards):
        ts, term, fr = T(s["ts"], torch.int64, dev), T(s["terminal"], torch.int32, dev), T(s["fraud"], torch.uint8, dev)
        owner = K.owner_keys(term, world)
        perm, seg = K.rekey(owner, world)
        rec = K.exchange_pack(ts, term, fr, perm).cpu().numpy()
        p = perm.cpu().numpy()
        np.testing.assert_array_equal(rec[:, 0], s["ts"][p])
        np.testing.assert_array_equal(rec[:, 1] >> 32, s["terminal"][p])
        np.testing.assert_array_equal((rec[:, 1] >> 31) & 1, s["fraud"][p])
        np.testing.assert_array_equal(rec[:, 1] & 0x7FFFFFFF, p)
        sent.append((rec, seg.cpu().numpy(), p))
    # host all-to-all: owner o receives source ranks' blocks in rank order
    replies = {}
    W = 3
    for o_ in range(world):
        blocks = [sent[r][0][sent[r][1][o_]:sent[r][1][o_ + 1]] for r in range(world)]
        recv = np.concatenate(blocks)
        rts, rterm, rfr = K.exchange_unpack(T(recv, torch.int64, dev), world)
        np.testing.assert_array_equal(rterm.cpu().numpy(), (recv[:, 1] >> 32) // world)
        rec = K.terminal_records_rekey(rts, rterm, rfr, (n_terms + world - 1) // world, 7, (1, 7, 30)).cpu().numpy()
        assert rec.shape == (len(recv), W)
        off = 0
        for r in range(world):
            replies.setdefault(r, {})[o_] = rec[off:off + len(blocks[r])]
            off += len(blocks[r])
    # host all-to-all back, then the reply assembly on each source rank
    for r, s in enumerate(shards):
        back = np.concatenate([replies[r][o_] for o_ in range(world)])
        X = torch.zeros((len(s["ts"]), 16), dtype=torch.float64, device=dev)
        K.reply_assemble(T(back, torch.int64, dev), T(sent[r][2], torch.int32, dev), W, X, 3 + 2 * W)
        got = X.cpu().numpy()[:, 9:15]
        rows = [ref_row[int(g)] for g in s["gid"]]
        np.testing.assert_array_equal(got, ref[rows][:, 9:15])


def test_deployed_model_rank_layout_v2(dev):
    """The reference's deployed RandomForestClassifier(random_state=0) -- 100 unlimited-depth
    trees, 1.68M nodes, up to 96k distinct thresholds on one feature (model_training.ipynb:2212,
    served at fraud_detection.py:81-82, :190-193) -- on the GPU through rank layout v2: the
    66,452-row test set of the notebook's split bit for bit against sklearn, both columns, then
    1M rows resampled from it (the all-chunks-at-once path for small batches and the
    chunk-sequential path for large ones)."""
    import ctypes

    z = np.load(os.path.join(ROOT, "bench_assets", "rf_deployed.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    lay, ns = ctypes.c_int32(), ctypes.c_int32()
    _lib.load().fdx_forest_layout(forest._h, ctypes.byref(lay), ctypes.byref(ns))
    assert lay.value == 2 and 16 <= ns.value <= 32
    X = z["test_X"]
    assert len(X) == 66_452
    np.testing.assert_array_equal(forest.predict(T(X, torch.float64, dev)).cpu().numpy(), z["test_proba1"])
    f0 = ops.Forest(dict(arrays, value1=z["value0"]), 15, z["mean"], z["scale"])
    np.testing.assert_array_equal(f0.predict(T(X, torch.float64, dev)).cpu().numpy(), z["test_proba0"])
    idx = np.random.default_rng(3).integers(0, len(X), 1_000_000)
    Xd = T(X, torch.float64, dev)[T(idx, torch.int64, dev)]
    got = forest.predict(Xd, ws=ops.workspace(forest.workspace_size(len(idx)), dev)).cpu().numpy()
    np.testing.assert_array_equal(got, z["test_proba1"][idx])


def test_deployed_model_20m_rows(dev):
    """The deployed model (RF(100, unlimited depth), model_training.ipynb:2212) at the size of
    bench_forest.py's line: 20M rows resampled from the notebook's 66,452 test rows, every row
    against sklearn's saved predict_proba[:, 1]."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf_deployed.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    X = z["test_X"]
    n = 20_000_000
    idx = _resampled(n, len(X), 11, dev)
    Xd = T(X, torch.float64, dev)[idx]
    got = forest.predict(Xd, ws=ops.workspace(forest.workspace_size(n), dev))
    del Xd
    want = T(z["test_proba1"], torch.float64, dev)[idx]
    bad = int((got != want).sum())
    assert bad == 0, f"{bad} of {n} rows differ from sklearn"


@pytest.mark.parametrize("base,n_c", [(375_000, 125_000), (0, 500_000)], ids=["rank3of8", "rank0of2"])
def test_config4_one_rank_shard(dev, base, n_c):
    """configs[3] (1M customers / 2M terminals / 365 days) as ONE rank sees it: rank 3 of 8
    owns customers [375000, 500000) and all their rows (~88M tx; the terminal ids range over
    all 2M); rank 0 of 2 (bench.py --gpus 2, strong scaling) owns [0, 500000), ~350M tx --
    every 8-byte column and the 32-byte scoring rows then span more than 2^31 bytes, so any
    32-bit offset arithmetic in a kernel would show here.  The sharded path (world 1 process group: its re-key exchange, owner-side
    records and reply assembly run through RCCL to self) must give the probabilities of the
    single-GPU fused path on the re-based ids on every row, and the sampled customers' and
    terminals' features must equal the C oracle's."""
    import socket

    import torch.distributed as dist

    from fdx.distributed import ShardedPipeline

    n_t = 2_000_000
    arrays, z = _model()
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    g = synth.generate_device(n_c, n_t, 365, seed=77, customer_offset=base, device=dev)
    n = g["ts"].numel()
    assert n > 480 * n_c
    args = (g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"])
    pipe = FraudPipeline(forest=forest)
    ws = ops.workspace(forest.workspace_size(n * 11 // 10), dev)
    p_single = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(args[0], args[1] - base, *args[2:], n_c, n_t, p_single, ws)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sp = ShardedPipeline(pipe, world=1, rank=0, n_terminals_total=n_t, customer_base=base, n_customers_local=n_c)
        p_shard = torch.zeros(n, dtype=torch.float64, device=dev)
        sp.run(*args, p_shard, ws)
        assert torch.equal(p_shard, p_single)
        X = sp.featurize(*args)
    finally:
        dist.destroy_process_group()
    d = {k: v.cpu().numpy() for k, v in g.items() if k in ("ts", "customer", "terminal", "amount", "fraud")}
    rng = np.random.default_rng(5)
    cust = rng.choice(n_c, 64, replace=False) + base
    term = rng.choice(n_t, 256, replace=False)
    for keys, col, cols, c0 in ((cust, "customer", CUST_COLS, 3), (term, "terminal", TERM_COLS, 9)):
        m = np.isin(d[col], keys)
        assert m.sum() > 1000
        f = oracle.featurize_arrays(d["ts"][m], d["customer"][m], d["terminal"][m], d["amount"][m], d["fraud"][m])
        rows = torch.from_numpy(np.flatnonzero(m)).to(dev)
        got = X[rows].cpu().numpy()
        for j, c in enumerate(cols):
            np.testing.assert_array_equal(got[:, c0 + j], f[c], err_msg=c)
        np.testing.assert_array_equal(p_single[rows].cpu().numpy(),
                                      oracle.forest_predict(got, arrays, z["mean"], z["scale"]))
