"""World-size-2 gloo test of the multi-GPU routing (fdx.distributed) on CPU.

The exchange code (owner keys, split exchange, all-to-all there and back, reply
reassembly) runs unchanged; only the per-rank kernels are replaced by numpy/oracle
stand-ins with the same record formats, so the test checks the distributed algorithm:
every rank's terminal features must equal the single-process oracle over the union of
all shards.  The HIP versions of the same kernels are covered by tests/test_gpu_*.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle


class CpuKernels:
    @staticmethod
    def owner_keys(term, world):
        return term % world

    @staticmethod
    def rekey(keys, n_keys):
        k = keys.numpy()
        perm = np.argsort(k, kind="stable").astype(np.int32)
        seg = np.r_[0, np.cumsum(np.bincount(k, minlength=n_keys))].astype(np.int64)
        return torch.from_numpy(perm), torch.from_numpy(seg)

    @staticmethod
    def gather(src, perm):
        return src[perm.long()]

    @staticmethod
    def argsort_i64(keys):
        return torch.from_numpy(np.argsort(keys.numpy(), kind="stable").astype(np.int32))

    @staticmethod
    def exchange_pack(ts, term, fraud, perm):
        p = perm.long()
        rec = torch.empty((len(p), 2), dtype=torch.int64)
        rec[:, 0] = ts[p]
        rec[:, 1] = (term[p].long() << 32) | ((fraud[p] != 0).long() << 31) | p
        return rec

    @staticmethod
    def exchange_unpack(rec, world):
        w = rec[:, 1]
        return rec[:, 0].clone(), ((w >> 32).int() // world).int(), ((w >> 31) & 1).to(torch.uint8)

    @staticmethod
    def terminal_windows(ts, fraud, seg, delay_days, windows_days):
        nb, risk = oracle.terminal_windows(ts.numpy(), fraud.numpy(), seg.numpy(), delay_days, windows_days)
        return torch.from_numpy(nb.astype(np.int32)), torch.from_numpy(risk)

    @staticmethod
    def terminal_records(ts, fraud, rows, seg, delay_days, windows_days):
        """count records (NB | FRAUD << 32) of grouped row q stored at rows[q]; segments may
        be out of time order (as the HIP kernel, each is time-sorted first, stably)"""
        r = rows.numpy()
        sg = seg.numpy()
        sid = np.repeat(np.arange(len(sg) - 1), np.diff(sg))
        r = r[np.lexsort((ts.numpy()[r], sid))]
        nb, risk = oracle.terminal_windows(ts.numpy()[r], fraud.numpy()[r], seg.numpy(), delay_days, windows_days)
        fr = np.rint(risk * nb).astype(np.int64)  # counts are small integers: exact
        rec = np.zeros((len(r), len(windows_days)), np.int64)
        rec[r] = (nb.astype(np.int64) | (fr << 32)).T
        return torch.from_numpy(rec)

    @staticmethod
    def terminal_records_rekey(rts, rterm, rfraud, n_local_terms, delay_days, windows_days, runs=True):
        perm, seg = CpuKernels.rekey(rterm, n_local_terms)
        return CpuKernels.terminal_records(rts, rfraud, perm, seg, delay_days, windows_days)

    @staticmethod
    def unpack_reply(back, W):
        b = back.numpy()
        nb = (b & 0xFFFFFFFF).astype(np.float64)
        fr = ((b >> 32) & 0xFFFFFFFF).astype(np.float64)
        with np.errstate(all="ignore"):
            risk = np.where(nb > 0, fr / np.maximum(nb, 1), 0.0)
        return nb, risk


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shards, n_terms, q, chunk_bytes=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fdx import distributed
    from fdx.distributed import exchange_terminal_features

    if chunk_bytes is not None:  # many point-to-point chunks per peer
        distributed.P2P_CHUNK_BYTES = chunk_bytes

    d = shards[rank]
    back, send_perm = exchange_terminal_features(
        CpuKernels, torch.from_numpy(d["ts"]), torch.from_numpy(d["terminal"]), torch.from_numpy(d["fraud"]),
        world, n_terms)
    nb, risk = CpuKernels.unpack_reply(back, 3)
    rows = send_perm.numpy()
    out_nb = np.zeros_like(nb); out_risk = np.zeros_like(risk)
    out_nb[rows] = nb; out_risk[rows] = risk
    q.put((rank, out_nb, out_risk))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk_bytes", [(2, None), (3, None), (3, 16 * 37)])
def test_terminal_exchange_matches_single_process(world, chunk_bytes):
    from fdx import synth

    n_terms = 150
    shards = [synth.generate(n_customers=120, n_terminals=n_terms, nb_days=60, r=30, seed=11 + r,
                             customer_offset=120 * r) for r in range(world)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shards, n_terms, q, chunk_bytes))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, nb, risk = q.get(timeout=120)
        res[r] = (nb, risk)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allc = {k: np.concatenate([s[k] for s in shards]) for k in shards[0]}
    order = np.argsort(allc["ts"], kind="stable")
    g = {k: v[order] for k, v in allc.items()}
    f = oracle.featurize_arrays(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"])
    inv = np.empty_like(order); inv[order] = np.arange(len(order))
    start = 0
    for r in range(world):
        n = len(shards[r]["ts"])
        idx = inv[start:start + n]
        start += n
        nb, risk = res[r]
        for k, w in enumerate((1, 7, 30)):
            np.testing.assert_array_equal(nb[:, k], f[f"TERMINAL_ID_NB_TX_{w}DAY_WINDOW"][idx])
            np.testing.assert_array_equal(risk[:, k], f[f"TERMINAL_ID_RISK_{w}DAY_WINDOW"][idx])


class NumpyStreamOwner:
    """Stand-in for the owner's incremental terminal state (fdx_stream_update, terminal half):
    keeps every local terminal's history and counts the delayed windows by brute force."""

    def __init__(self, windows_days=(1, 7, 30), delay_days=7):
        self.win = [w * 86400 * 10**9 for w in windows_days]
        self.delay = delay_days * 86400 * 10**9
        self.hist = {}

    def __call__(self, rts, rterm, rfr):
        ts, tl, fr = rts.numpy(), rterm.numpy(), rfr.numpy()
        rec = np.zeros((len(ts), len(self.win)), np.int64)
        for i in np.lexsort((np.arange(len(ts)), ts)):
            h = self.hist.setdefault(int(tl[i]), ([], []))
            ht, hf = np.array(h[0], np.int64), np.array(h[1], np.int64)
            t = int(ts[i])
            for k, w in enumerate(self.win):
                m = (ht <= t - self.delay) & (ht > t - self.delay - w)
                rec[i, k] = int(m.sum()) | (int(hf[m].sum()) << 32)
            h[0].append(t)
            h[1].append(int(fr[i]))
        return torch.from_numpy(rec)


def _stream_worker(rank, world, port, shards, cuts, n_terms, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fdx.streaming import stream_terminal_exchange

    d = shards[rank]
    owner = NumpyStreamOwner()
    nb_all, risk_all = np.zeros((len(d["ts"]), 3)), np.zeros((len(d["ts"]), 3))
    for a_t, b_t in zip(cuts[:-1], cuts[1:]):        # the same time cuts on every rank
        sel = np.flatnonzero((d["ts"] >= a_t) & (d["ts"] < b_t))
        back, send_perm = stream_terminal_exchange(
            CpuKernels, owner, torch.from_numpy(d["ts"][sel]), torch.from_numpy(d["terminal"][sel]),
            torch.from_numpy(d["fraud"][sel]), world, n_terms)
        nb, risk = CpuKernels.unpack_reply(back, 3)
        rows = sel[send_perm.numpy()]
        nb_all[rows], risk_all[rows] = nb, risk
    q.put((rank, nb_all, risk_all))
    dist.barrier()
    dist.destroy_process_group()


def test_stream_terminal_exchange_matches_single_process():
    """config 5 routing over 2 ranks: micro-batches cut at the same times on every rank, rows to
    their terminal's owner, the owner's incremental state, records back -- equal to the
    single-process terminal features of the whole history"""
    from fdx import synth

    world, n_terms = 2, 120
    shards = [synth.generate(n_customers=80, n_terminals=n_terms, nb_days=50, r=30, seed=21 + r,
                             customer_offset=80 * r) for r in range(world)]
    t0 = min(s["ts"].min() for s in shards)
    t1 = max(s["ts"].max() for s in shards) + 1
    cuts = np.unique(np.r_[t0, np.random.default_rng(4).integers(t0, t1, 25), t1])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, shards, cuts, n_terms, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, nb, risk = q.get(timeout=300)
        res[r] = (nb, risk)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allc = {k: np.concatenate([s[k] for s in shards]) for k in shards[0]}
    order = np.argsort(allc["ts"], kind="stable")
    g = {k: v[order] for k, v in allc.items()}
    f = oracle.featurize_arrays(g["ts"], g["customer"], g["terminal"], g["amount"], g["fraud"])
    inv = np.empty_like(order); inv[order] = np.arange(len(order))
    start = 0
    for r in range(world):
        n = len(shards[r]["ts"])
        idx = inv[start:start + n]
        start += n
        nb, risk = res[r]
        for k, w in enumerate((1, 7, 30)):
            np.testing.assert_array_equal(nb[:, k], f[f"TERMINAL_ID_NB_TX_{w}DAY_WINDOW"][idx])
            np.testing.assert_array_equal(risk[:, k], f[f"TERMINAL_ID_RISK_{w}DAY_WINDOW"][idx])


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
def test_customer_shards_cover_and_balance(world):
    """Contiguous customer ranges, balanced by tx count, every customer owned once -- also
    when the customer count does not divide by world (the round-1 n // world split left the
    remainder's ids outside every rank's range)."""
    from fdx.distributed import customer_shards

    rng = np.random.default_rng(world)
    for n_cust in (1, 7, 1001, 50_003):
        counts = rng.poisson(rng.uniform(0, 4, n_cust) * 183)
        sh = customer_shards(counts, world)
        assert len(sh) == world and sh[0][0] == 0
        assert all(sh[k][0] + sh[k][1] == sh[k + 1][0] for k in range(world - 1))
        assert sh[-1][0] + sh[-1][1] == n_cust and all(c >= 0 for _, c in sh)
        if n_cust >= 1000:
            rows = [int(counts[b:b + c].sum()) for b, c in sh]
            ideal = counts.sum() / world
            assert max(rows) - ideal <= counts.max() + 1, (rows, ideal)
