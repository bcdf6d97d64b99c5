"""BASELINE.json configs[4] on the GPU: streaming micro-batches of 64k CDC transactions over the
1M-customer / 2M-terminal window state (config 4's key space), incremental update + scoring.

  * world 1, the bench_stream.py workload: 38 days of history streamed day by day into the
    state, then day 38 as 64k-transaction micro-batches through StreamScorer (fused: state
    kernels -> NB / SUM planes + count records -> rank rows -> forest).  For 64 sampled
    customers and 64 sampled terminals (every day-38 row of them) the features the state
    kernels wrote must equal the C oracle run over the FULL history of those keys, and the
    scored probabilities must equal the oracle forest on the oracle's features.
  * world 4 and 8, host-simulated: ShardedStreamScorer's per-batch dataflow with every kernel
    on the GPU (the rank's customer state, owner keys / re-key / pack, the owner's
    fdx_stream_update on received rows, reply, row assembly, forest); only the two
    all-to-alls run on the host.  Every rank's probabilities must equal one StreamScorer over
    the union of the ranks' rows, batch by batch.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from fdx import ops, synth
from fdx.streaming import StreamScorer, StreamState

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DAY = 86_400 * 10**9


def _model():
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    return arrays, z["mean"], z["scale"]


def test_config5_64k_batches_over_1m_2m_state(dev):
    n_c, n_t, hist_days, batch = 1_000_000, 2_000_000, 38, 65_536
    g = synth.generate_device(n_c, n_t, hist_days + 1, seed=4321, device=dev)
    d = {k: g[k].cpu().numpy() for k in ("ts", "customer", "terminal", "amount", "fraud")}
    n = len(d["ts"])
    assert n > 60_000_000
    split = synth.START_NS + hist_days * DAY
    h = int(np.searchsorted(d["ts"], split))
    day_cuts = np.searchsorted(d["ts"][:h], synth.START_NS + np.arange(hist_days + 1) * DAY)
    day_cuts[-1] = h
    mb = np.r_[np.arange(h, n, batch), n]
    arrays, mean, scale = _model()
    forest = ops.Forest(arrays, 15, mean, scale)
    cap = int(max(np.diff(day_cuts).max(), batch))
    sc = StreamScorer(forest, n_c, n_t, max_batch=cap)
    cols = (("ts", torch.int64), ("customer", torch.int32), ("amount", torch.float64), ("terminal", torch.int32),
            ("fraud", torch.uint8))

    def run(a, b):
        return sc.score(*(g[k][a:b] for k, _ in cols))

    for k in range(hist_days):
        run(int(day_cuts[k]), int(day_cuts[k + 1]))
    sc.state.check()
    # sampled keys with rows on the streamed day
    rng = np.random.default_rng(11)
    s_cust = rng.choice(np.unique(d["customer"][h:]), 64, replace=False)
    s_term = rng.choice(np.unique(d["terminal"][h:]), 64, replace=False)
    want_c = np.isin(d["customer"][h:], s_cust)
    want_t = np.isin(d["terminal"][h:], s_term)
    # features (from the fused planes / records) and probabilities of the sampled day-38 rows
    got_X = np.full((n - h, 15), np.nan)
    got_p = np.full(n - h, np.nan)
    for a, b in zip(mb[:-1], mb[1:]):
        p = run(int(a), int(b)).cpu().numpy()
        m = b - a
        sel = np.flatnonzero(want_c[a - h:b - h] | want_t[a - h:b - h])
        if len(sel) == 0:
            continue
        cnb = sc.cnb[:3 * m].view(3, m).cpu().numpy()
        csum = sc.csum[:3 * m].view(3, m).cpu().numpy()
        trec = sc.trec[:m * 3].view(m, 3).cpu().numpy()
        rows = sel + (a - h)
        got_p[rows] = p[sel]
        for w in range(3):
            got_X[rows, 3 + 2 * w] = cnb[w, sel]
            got_X[rows, 4 + 2 * w] = csum[w, sel] / cnb[w, sel]
            nb_t = trec[sel, w] & 0xFFFFFFFF
            fr_t = trec[sel, w] >> 32
            got_X[rows, 9 + 2 * w] = nb_t
            got_X[rows, 10 + 2 * w] = np.where(nb_t > 0, fr_t / np.maximum(nb_t, 1), 0.0)
    sc.finish()
    # the oracle over the FULL history of the sampled keys (and of the terminals / customers
    # the sampled rows touch, for the probabilities)
    rows_c = np.flatnonzero(want_c) + h
    rows_t = np.flatnonzero(want_t) + h
    rows = np.union1d(rows_c, rows_t)
    need_c = np.isin(d["customer"], np.unique(d["customer"][rows]))
    need_t = np.isin(d["terminal"], np.unique(d["terminal"][rows]))
    fc = oracle.featurize_arrays(*(d[k][need_c] for k in ("ts", "customer", "terminal", "amount", "fraud")))
    ft = oracle.featurize_arrays(*(d[k][need_t] for k in ("ts", "customer", "terminal", "amount", "fraud")))
    ic, it = np.full(n, -1), np.full(n, -1)
    ic[np.flatnonzero(need_c)] = np.arange(need_c.sum())
    it[np.flatnonzero(need_t)] = np.arange(need_t.sum())
    Xo = np.column_stack([d["amount"][rows], oracle.weekend_flag(d["ts"][rows]), oracle.night_flag(d["ts"][rows])]
                         + [fc[c][ic[rows]] for c in oracle.CUSTOMER_COLS]
                         + [ft[c][it[rows]] for c in oracle.TERMINAL_COLS])
    g_rows = rows - h
    for j in range(3, 9):  # customer features of the sampled customers' rows
        sel = np.isin(rows, rows_c)
        np.testing.assert_array_equal(got_X[g_rows[sel], j], Xo[sel, j], err_msg=oracle.INPUT_FEATURES[j])
    for j in range(9, 15):  # terminal features of the sampled terminals' rows
        sel = np.isin(rows, rows_t)
        np.testing.assert_array_equal(got_X[g_rows[sel], j], Xo[sel, j], err_msg=oracle.INPUT_FEATURES[j])
    np.testing.assert_array_equal(got_p[g_rows], oracle.forest_predict(Xo, arrays, mean, scale))
    assert len(rows_c) >= 64 and len(rows_t) >= 64


@pytest.mark.parametrize("world", [4, 8])
def test_sharded_stream_world_gt1_host_simulated(dev, world):
    """ShardedStreamScorer.score's dataflow for `world` ranks on one GPU, all-to-alls on the
    host; every kernel (customer state, exchange pack / unpack, owner fdx_stream_update,
    reply assembly, forest) is the HIP one."""
    from fdx import _lib
    from fdx.distributed import GpuKernels as K

    C, n_terms, days, batch = 400, 900, 50, 4_096
    arrays, mean, scale = _model()
    forest = ops.Forest(arrays, 15, mean, scale)
    shards = [synth.generate(C, n_terms, days, r=20, seed=90 + r, customer_offset=C * r) for r in range(world)]
    whole = {k: np.concatenate([s[k] for s in shards]) for k in ("ts", "customer", "terminal", "amount", "fraud")}
    whole["rank"] = np.concatenate([np.full(len(s["ts"]), r) for r, s in enumerate(shards)])
    whole["pos"] = np.concatenate([np.arange(len(s["ts"])) for s in shards])
    o = np.argsort(whole["ts"], kind="stable")
    whole = {k: v[o] for k, v in whole.items()}
    N = len(whole["ts"])
    cuts = np.r_[np.arange(0, N, batch), N]
    T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    ref = StreamScorer(forest, C * world, n_terms, terminal_ring=1024, max_batch=batch)
    n_tl = (n_terms + world - 1) // world
    states = [StreamState(C, n_tl, terminal_ring=1024, max_batch=batch * world) for _ in range(world)]
    ws = ops.workspace(forest.workspace_size_max(batch), dev)
    checked = 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        exp = ref.score(T(whole["ts"][a:b], torch.int64), T(whole["customer"][a:b], torch.int32),
                        T(whole["amount"][a:b], torch.float64), T(whole["terminal"][a:b], torch.int32),
                        T(whole["fraud"][a:b], torch.uint8)).cpu().numpy()
        part = []
        for r in range(world):  # phase 1: customer half + owner re-key + pack
            m = whole["rank"][a:b] == r
            ts, cu = T(whole["ts"][a:b][m], torch.int64), T(whole["customer"][a:b][m] - C * r, torch.int32)
            am, te = T(whole["amount"][a:b][m], torch.float64), T(whole["terminal"][a:b][m], torch.int32)
            fr = T(whole["fraud"][a:b][m], torch.uint8)
            nr = ts.numel()
            cnb = torch.empty((3, nr), dtype=torch.int32, device=dev)
            csum = torch.empty((3, nr), dtype=torch.float64, device=dev)
            if nr:
                states[r].update(ts, cu, am, cust_nb=cnb, cust_sum=csum)
            perm, seg = K.rekey(K.owner_keys(te, world), world)
            rec = K.exchange_pack(ts, te, fr, perm).cpu().numpy() if nr else np.zeros((0, 2), np.int64)
            part.append(dict(ts=ts, am=am, cnb=cnb, csum=csum, perm=perm, seg=seg.cpu().numpy(), rec=rec,
                             sel=np.flatnonzero(m), n=nr))
        replies = {}
        for o_ in range(world):  # host all-to-all; owner-side incremental terminal update
            blocks = [p["rec"][p["seg"][o_]:p["seg"][o_ + 1]] for p in part]
            recv = np.concatenate(blocks)
            if len(recv):
                rts, rterm, rfr = K.exchange_unpack(T(recv, torch.int64), world)
                rr = torch.empty((len(recv), 3), dtype=torch.int64, device=dev)
                states[o_].update(rts, terminal=rterm, fraud=rfr, term_records=rr)
                rr = rr.cpu().numpy()
            else:
                rr = np.zeros((0, 3), np.int64)
            off = 0
            for r, blk in enumerate(blocks):
                replies.setdefault(r, []).append(rr[off:off + len(blk)])
                off += len(blk)
        for r, p in enumerate(part):  # host all-to-all back; rank r assembles and scores
            if p["n"] == 0:
                continue
            back = T(np.concatenate(replies[r]), torch.int64)
            inv = ops.invert_perm(p["perm"])
            ops.forest_prepare_grouped(forest, _lib.FDX_FLAGS_NOTEBOOK, p["ts"], p["am"], p["cnb"], p["csum"], None,
                                       inv, back, ws, n=p["n"], val_is_sum=True)
            out = torch.empty(p["n"], dtype=torch.float64, device=dev)
            ops.forest_traverse(forest, p["n"], ws, out)
            np.testing.assert_array_equal(out.cpu().numpy(), exp[p["sel"]])
            checked += p["n"]
    for s in states:
        s.check()
    ref.finish()
    assert checked == N
