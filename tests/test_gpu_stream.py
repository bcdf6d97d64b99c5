"""Config 5 streaming engine (csrc/fdx_stream.hip, fdx.streaming) on the GPU.

Feeding a history micro-batch by micro-batch must give the features of the batch path over
the whole history, bit for bit: against the reference's own outputs on the golden frame
(tests/golden/tiny_a.npz, produced by feature_transformation.ipynb's functions) and against
the oracle on synthetic streams with ties, bursts of one key inside a batch and other
window / delay settings.  Then: scoring equals the forest on the batch features, the sharded
scorer (RCCL world 1) equals the single-GPU one, and state errors are reported."""
import os
import socket

import numpy as np
import pytest
import torch

import oracle
from fdx import _lib, ops
from fdx.streaming import ShardedStreamScorer, StreamScorer, StreamState

pytestmark = pytest.mark.gpu

FEATS = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + oracle.CUSTOMER_COLS + oracle.TERMINAL_COLS


def T(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)


def _stream(state, cols, dev, cuts, X=None):
    n = len(cols["ts"])
    out = np.empty((n, 3 + 4 * state.W))
    for a, b in zip(cuts[:-1], cuts[1:]):
        x = state.update(T(cols["ts"][a:b], torch.int64, dev), T(cols["customer"][a:b], torch.int32, dev),
                         T(cols["amount"][a:b], torch.float64, dev), T(cols["terminal"][a:b], torch.int32, dev),
                         T(cols["fraud"][a:b], torch.uint8, dev))
        out[a:b] = x.cpu().numpy()
    state.check()
    return out


def _golden_cols(golden):
    z = golden("tiny_a.npz")
    o = np.argsort(z["TRANSACTION_ID"], kind="stable")
    g = {k: z[k][o] for k in z.files}
    cols = {"ts": g["TX_DATETIME"], "customer": g["CUSTOMER_ID"], "terminal": g["TERMINAL_ID"],
            "amount": g["TX_AMOUNT"], "fraud": g["TX_FRAUD"]}
    return g, cols


@pytest.mark.parametrize("batch", [1, 7, 333, 4096, 1 << 20])
def test_stream_matches_reference_golden(dev, golden, batch):
    g, cols = _golden_cols(golden)
    n = len(cols["ts"])
    st = StreamState(int(cols["customer"].max()) + 1, int(cols["terminal"].max()) + 1, max_batch=min(batch, n))
    X = _stream(st, cols, dev, list(range(0, n, batch)) + [n])
    for j, c in enumerate(FEATS):
        np.testing.assert_array_equal(X[:, j], g[c].astype(np.float64), err_msg=c)


@pytest.mark.parametrize("batch", [1000, 1 << 20])
def test_stream_planes_match_reference_golden(dev, golden, batch):
    """The scoring-layout outputs (NB / SUM planes, count records; no X matrix) hold the same
    features: NB_w, SUM_w / NB_w = AVG_w, FRAUD_w / NB_w = RISK_w (0 when NB_w = 0)."""
    g, cols = _golden_cols(golden)
    n = len(cols["ts"])
    st = StreamState(int(cols["customer"].max()) + 1, int(cols["terminal"].max()) + 1, max_batch=min(batch, n))
    W = st.W
    nb, sm, rec = np.empty((W, n), np.int32), np.empty((W, n)), np.empty((n, W), np.int64)
    for a in range(0, n, batch):
        b = min(a + batch, n)
        m = b - a
        cnb = torch.empty((W, m), dtype=torch.int32, device=dev)
        csum = torch.empty((W, m), dtype=torch.float64, device=dev)
        trec = torch.empty((m, W), dtype=torch.int64, device=dev)
        x = st.update(T(cols["ts"][a:b], torch.int64, dev), T(cols["customer"][a:b], torch.int32, dev),
                      T(cols["amount"][a:b], torch.float64, dev), T(cols["terminal"][a:b], torch.int32, dev),
                      T(cols["fraud"][a:b], torch.uint8, dev), term_records=trec, cust_nb=cnb, cust_sum=csum)
        assert x is None
        nb[:, a:b], sm[:, a:b], rec[a:b] = cnb.cpu().numpy(), csum.cpu().numpy(), trec.cpu().numpy()
    st.check()
    tnb, tfr = rec & 0xFFFFFFFF, rec >> 32
    for w, d in enumerate((1, 7, 30)):
        np.testing.assert_array_equal(nb[w], g[f"CUSTOMER_ID_NB_TX_{d}DAY_WINDOW"])
        np.testing.assert_array_equal(sm[w] / nb[w], g[f"CUSTOMER_ID_AVG_AMOUNT_{d}DAY_WINDOW"])
        np.testing.assert_array_equal(tnb[:, w], g[f"TERMINAL_ID_NB_TX_{d}DAY_WINDOW"])
        with np.errstate(invalid="ignore", divide="ignore"):
            risk = np.where(tnb[:, w] > 0, tfr[:, w] / tnb[:, w], 0.0)
        np.testing.assert_array_equal(risk, g[f"TERMINAL_ID_RISK_{d}DAY_WINDOW"])


@pytest.mark.parametrize("windows,delay,seed", [((1, 7, 30), 7, 0), ((2, 5), 3, 1), ((3,), 1, 2),
                                                ((1, 2, 4, 8, 16, 32), 7, 3)])
def test_stream_random_batches_vs_oracle(dev, windows, delay, seed):
    """ties inside and across batches, 50-row bursts of one customer inside a batch, random
    batch boundaries, other window / delay settings"""
    rng = np.random.default_rng(seed)
    n, n_c, n_t = 30_000, 300, 200
    ts = np.sort(rng.integers(0, 90 * 86400, n)) * 1_000_000_000 + 1_717_200_000_000_000_000
    ts[1000:1100] = ts[1000]                          # a tie run across a batch cut
    cust = rng.integers(0, n_c, n).astype(np.int32)
    cust[5000:5050] = 17                              # a burst of one key
    term = rng.integers(0, n_t, n).astype(np.int32)
    amt = np.round(rng.uniform(0, 100, n), 2)
    amt[7000:7040] = 12.5                             # equal values (pandas' n_same rule)
    fr = (rng.random(n) < 0.1).astype(np.uint8)
    cols = {"ts": ts, "customer": cust, "terminal": term, "amount": amt, "fraud": fr}
    cuts = np.unique(np.r_[0, np.sort(rng.integers(0, n, 60)), 1050, 5020, n])
    st = StreamState(n_c, n_t, windows, delay, customer_ring=1024, terminal_ring=2048,
                     max_batch=int(np.diff(cuts).max()))
    X = _stream(st, cols, dev, list(cuts))
    f = oracle.featurize_arrays(ts, cust, term, amt, fr, windows, delay)
    W = len(windows)
    for k, w in enumerate(windows):
        np.testing.assert_array_equal(X[:, 3 + 2 * k], f[f"CUSTOMER_ID_NB_TX_{w}DAY_WINDOW"])
        np.testing.assert_array_equal(X[:, 4 + 2 * k], f[f"CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW"])
        np.testing.assert_array_equal(X[:, 3 + 2 * W + 2 * k], f[f"TERMINAL_ID_NB_TX_{w}DAY_WINDOW"])
        np.testing.assert_array_equal(X[:, 4 + 2 * W + 2 * k], f[f"TERMINAL_ID_RISK_{w}DAY_WINDOW"])
    np.testing.assert_array_equal(X[:, 1], oracle.weekend_flag(ts))
    np.testing.assert_array_equal(X[:, 2], oracle.night_flag(ts))


def test_stream_spark_flags_and_reset(dev, golden):
    g, cols = _golden_cols(golden)
    n = len(cols["ts"])
    st = StreamState(int(cols["customer"].max()) + 1, int(cols["terminal"].max()) + 1, max_batch=n,
                     flags_mode=_lib.FDX_FLAGS_SPARK)
    X1 = _stream(st, cols, dev, [0, n])
    np.testing.assert_array_equal(X1[:, 1], oracle.spark_weekend_flag(cols["ts"]))
    np.testing.assert_array_equal(X1[:, 2], oracle.spark_night_flag(cols["ts"]))
    st.reset()
    X2 = _stream(st, cols, dev, [0, 5000, n])
    np.testing.assert_array_equal(X2, X1)


def test_stream_state_errors_reported(dev):
    base = 1_717_200_000_000_000_000
    day = 86400 * 10**9
    st = StreamState(4, 4, customer_ring=4, terminal_ring=4, max_batch=64)
    ts = base + np.arange(10, dtype=np.int64) * 3_600 * 10**9      # 10 rows of one key within a day
    z = np.zeros(10, np.int32)
    args = lambda t, c, k: (T(t, torch.int64, dev), T(c, torch.int32, dev), T(np.ones(len(t)), torch.float64, dev),  # noqa: E731
                            T(k, torch.int32, dev), T(np.zeros(len(t)), torch.uint8, dev))
    st.update(*args(ts, z, z))
    with pytest.raises(_lib.FdxUnsupported, match="customer ring overflow"):
        st.check()
    st.reset()
    st.update(*args(ts[:2], z[:2] + 9, z[:2]))
    with pytest.raises(_lib.FdxUnsupported, match="outside"):
        st.check()
    st.reset()
    st.update(*args(ts[5:6], z[:1], z[:1]))
    st.update(*args(ts[:1], z[:1], z[:1]))
    with pytest.raises(_lib.FdxUnsupported, match="back in time"):
        st.check()
    st.reset()
    st.update(*args(ts[:3] + 40 * day, z[:3], z[:3] + 1))                  # fine again after reset
    st.check()


def _forest(golden):
    z = golden("forest_rf5d8.npz")
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1", "node_offsets")}
    return ops.Forest(arrays, 15, z["mean"], z["scale"])


@pytest.mark.parametrize("fused", [True, False])
def test_stream_scorer_equals_batch_scoring(dev, golden, fused):
    g, cols = _golden_cols(golden)
    n = len(cols["ts"])
    forest = _forest(golden)
    sc = StreamScorer(forest, int(cols["customer"].max()) + 1, int(cols["terminal"].max()) + 1, max_batch=2048,
                      fused=fused)
    got = np.empty(n)
    for a in range(0, n, 2048):
        b = min(a + 2048, n)
        p = sc.score(*(T(cols[k][a:b], dt, dev) for k, dt in (("ts", torch.int64), ("customer", torch.int32),
                                                              ("amount", torch.float64), ("terminal", torch.int32),
                                                              ("fraud", torch.uint8))))
        got[a:b] = p.cpu().numpy()
    sc.state.check()
    Xg = np.stack([g[c].astype(np.float64) for c in FEATS], axis=1)
    ref = forest.predict(T(Xg, torch.float64, dev)).cpu().numpy()
    np.testing.assert_array_equal(got, ref)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_stream_world1_equals_single(dev, golden):
    import torch.distributed as dist

    g, cols = _golden_cols(golden)
    n = len(cols["ts"])
    forest = _forest(golden)
    n_c, n_t = int(cols["customer"].max()) + 1, int(cols["terminal"].max()) + 1
    single = StreamScorer(forest, n_c, n_t, max_batch=3000)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sh = ShardedStreamScorer(forest, world=1, rank=0, n_customers_local=n_c, customer_base=0,
                                 n_terminals_total=n_t, max_batch=3000)
        for a in range(0, n, 3000):
            b = min(a + 3000, n)
            args = [T(cols[k][a:b], dt, dev) for k, dt in (("ts", torch.int64), ("customer", torch.int32),
                                                            ("amount", torch.float64), ("terminal", torch.int32),
                                                            ("fraud", torch.uint8))]
            p1 = single.score(*args).cpu().numpy()
            p2 = sh.score(*args).cpu().numpy()
            np.testing.assert_array_equal(p2, p1)
        sh.state.check()
    finally:
        dist.destroy_process_group()


def test_stream_scorer_raises_without_explicit_check(dev, golden):
    """StreamScorer.score watches the status bits itself: a ring overflow in one batch makes
    the next score() (or finish()) raise, with no state.check() by the caller."""
    forest = _forest(golden)
    sc = StreamScorer(forest, 4, 4, customer_ring=4, terminal_ring=4, max_batch=64)
    base = 1_717_200_000_000_000_000
    ts = base + np.arange(10, dtype=np.int64) * 3_600 * 10**9   # 10 rows of one key: ring of 4 overflows
    z = np.zeros(10, np.int32)
    args = (T(ts, torch.int64, dev), T(z, torch.int32, dev), T(np.ones(10), torch.float64, dev),
            T(z, torch.int32, dev), T(np.zeros(10), torch.uint8, dev))
    sc.score(*args)
    with pytest.raises(_lib.FdxUnsupported, match="ring overflow"):
        sc.finish()


def test_stream_scorer_graph_equals_score(dev, golden):
    """score_graph (one HIP graph per batch size: the state update, row assembly, forest walk,
    status copy and the probabilities' copy to pinned host memory) == score(), batch for batch:
    inputs staged through one device buffer (fixed addresses), a ragged last batch (a second
    graph), one size captured before use; and a ring overflow in a graphed batch still raises."""
    g, cols = _golden_cols(golden)
    n = len(cols["ts"])
    forest = _forest(golden)
    n_c, n_t = int(cols["customer"].max()) + 1, int(cols["terminal"].max()) + 1
    ref_sc = StreamScorer(forest, n_c, n_t, max_batch=2048)
    sc = StreamScorer(forest, n_c, n_t, max_batch=2048)
    keys = (("ts", torch.int64), ("customer", torch.int32), ("amount", torch.float64), ("terminal", torch.int32),
            ("fraud", torch.uint8))
    stage = {k: torch.empty(2048, dtype=dt, device=dev) for k, dt in keys}
    out_h = torch.empty(2048, dtype=torch.float64).pin_memory()
    sc.score_graph(*(stage[k][:2048] for k, _ in keys), out_host=out_h, replay=False)
    for a in range(0, n, 2048):
        b = min(a + 2048, n)
        args = [T(cols[k][a:b], dt, dev) for k, dt in keys]
        want = ref_sc.score(*args).cpu().numpy()
        for (k, _), t in zip(keys, args):
            stage[k][:b - a].copy_(t)
        p = sc.score_graph(*(stage[k][:b - a] for k, _ in keys), out_host=out_h)
        torch.cuda.current_stream().synchronize()
        np.testing.assert_array_equal(p.cpu().numpy(), want)
        np.testing.assert_array_equal(out_h[:b - a].numpy(), want)
    assert len(sc._graphs) == (1 if n % 2048 == 0 else 2)
    sc.finish()
    # a forest whose layout changed (set_variant re-lays its device buffers) is captured again:
    # the old graphs held the freed buffers' addresses
    forest.set_variant(0)
    sc2 = StreamScorer(forest, n_c, n_t, max_batch=2048)
    ref2 = StreamScorer(forest, n_c, n_t, max_batch=2048)
    args = [T(cols[k][:2048], dt, dev) for k, dt in keys]
    for (k, _), t in zip(keys, args):
        stage[k][:2048].copy_(t)
    sc2.score_graph(*(stage[k][:2048] for k, _ in keys), out_host=out_h, replay=False)
    forest.set_variant(forest.variant if forest.variant != 0 else 1)
    p2 = sc2.score_graph(*(stage[k][:2048] for k, _ in keys), out_host=out_h).cpu().numpy()
    np.testing.assert_array_equal(p2, ref2.score(*args).cpu().numpy())
    assert len(sc2._graphs) == 1
    small = StreamScorer(forest, 4, 4, customer_ring=4, terminal_ring=4, max_batch=64)
    base = 1_717_200_000_000_000_000
    ts = base + np.arange(10, dtype=np.int64) * 3_600 * 10**9
    z = np.zeros(10, np.int32)
    small.score_graph(T(ts, torch.int64, dev), T(z, torch.int32, dev), T(np.ones(10), torch.float64, dev),
                      T(z, torch.int32, dev), T(np.zeros(10), torch.uint8, dev))
    with pytest.raises(_lib.FdxUnsupported, match="ring overflow"):
        small.finish()
