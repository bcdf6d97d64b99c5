"""The multi-GPU path's HIP kernels and RCCL calls on one GPU (world_size 1): the sharded
pipeline (owner keys, exchange pack/unpack, all-to-all to self, reply pack/assemble) must
give the same feature matrix, bit for bit, as the single-GPU pipeline.  world > 1 routing
is covered on CPU by tests/test_distributed_cpu.py (gloo, world 2 and 3)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from fdx import ops, synth
from fdx.distributed import ShardedPipeline
from fdx.pipeline import FraudPipeline

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_pipeline_world1_matches_single(dev):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        d = synth.generate(n_customers=3000, n_terminals=5000, nb_days=90, seed=3, customer_offset=0)
        T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
        args = (T(d["ts"], torch.int64), T(d["customer"], torch.int32), T(d["terminal"], torch.int32),
                T(d["amount"], torch.float64), T(d["fraud"], torch.uint8))
        pipe = FraudPipeline()
        ref = pipe.featurize(*args, 3000, 5000).X.cpu().numpy()
        sp = ShardedPipeline(pipe, world=1, rank=0, n_terminals_total=5000, customer_base=0, n_customers_local=3000)
        got = sp.featurize(*args).cpu().numpy()
        np.testing.assert_array_equal(got, ref)
        # exchange kernels with world > 1 semantics (owner = t % 4, local id = t / 4)
        own = ops.key_map(args[2], 0, 4).cpu().numpy()
        np.testing.assert_array_equal(own, d["terminal"] % 4)
        np.testing.assert_array_equal(ops.key_map(args[2], 1, 4).cpu().numpy(), d["terminal"] // 4)
        np.testing.assert_array_equal(ops.key_map(args[1], 2, 7).cpu().numpy(), d["customer"] - 7)
    finally:
        dist.destroy_process_group()


def test_fused_scoring_paths_agree(dev, golden):
    """run_fused (z32 written by the window outputs) == featurize + float64 X + predict, and
    the sharded run (world 1) gives the same probabilities."""
    z = golden("forest_rf5d8.npz")
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1",
                                "node_offsets")}
    forest = ops.Forest(arrays, 15, z["mean"], z["scale"])
    d = synth.generate(n_customers=2000, n_terminals=4000, nb_days=60, seed=9)
    T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
    args = (T(d["ts"], torch.int64), T(d["customer"], torch.int32), T(d["terminal"], torch.int32),
            T(d["amount"], torch.float64), T(d["fraud"], torch.uint8))
    n = len(d["ts"])
    pipe = FraudPipeline(forest=forest)
    _, p_ref = pipe.run(*args, 2000, 4000)
    ws = ops.workspace(forest.workspace_size(n), dev)
    p1 = torch.empty(n, dtype=torch.float64, device=dev)
    pipe.run_fused(*args, 2000, 4000, p1, ws)
    np.testing.assert_array_equal(p1.cpu().numpy(), p_ref.cpu().numpy())
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sp = ShardedPipeline(pipe, world=1, rank=0, n_terminals_total=4000, customer_base=0, n_customers_local=2000)
        p2 = torch.zeros(n, dtype=torch.float64, device=dev)
        sp.run(*args, p2, ws)
        np.testing.assert_array_equal(p2.cpu().numpy(), p_ref.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("parts", [1, 4, 8, 100])
def test_terminal_records_unsorted_runs(dev, parts):
    """The owner side of the exchange: rows arrive as one time-sorted run per source rank,
    so a stable re-key by terminal yields segments of concatenated runs.  The records of
    fdx_terminal_windows_grouped(runs = 1) over them must equal those of the time-sorted input
    row by row -- for 1 run (sorted), a few runs, and more runs than the per-run search handles
    (100 > kMaxRuns: direct counts)."""
    d = synth.generate(n_customers=600, n_terminals=300, nb_days=80, r=30, seed=5)
    T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
    n = len(d["ts"])
    ts, term, fr = T(d["ts"], torch.int64), T(d["terminal"], torch.int32), T(d["fraud"], torch.uint8)
    tperm, tseg, tgts, _ = ops.rekey_payload(term, 300, ts, flag=fr)
    ref = ops.terminal_windows_grouped(tgts, tseg, rows=tperm).cpu().numpy()   # by input row
    # "receive buffer": rows grouped by source part (customer % parts), time order inside
    order = np.argsort(d["customer"] % parts, kind="stable")
    rts, rterm, rfr = T(d["ts"][order], torch.int64), T(d["terminal"][order], torch.int32), \
        T(d["fraud"][order], torch.uint8)
    gperm, gseg, gts, _ = ops.rekey_payload(rterm, 300, rts, flag=rfr)
    got = ops.terminal_windows_grouped(gts, gseg, rows=gperm, runs=True).cpu().numpy()  # by receive index
    np.testing.assert_array_equal(got, ref[order])
    assert n > 0


@pytest.mark.parametrize("parts", [8, 100, 2500])
def test_terminal_records_hot_terminals_long_segments(dev, parts):
    """Segments far longer than the LDS stage (8 terminals, ~9k rows each): the global-memory
    path of k_terminal_g -- prefix fraud counts in scratch, binary searches per run -- for 8
    and 100 runs, and the direct count past the long run list (2,500 runs > 2,047).  The
    records must equal the time-sorted input's row by row, and the oracle's on one terminal."""
    import oracle

    d = synth.generate(n_customers=2500, n_terminals=8, nb_days=15, r=200, seed=21)
    T = lambda a, t: torch.from_numpy(np.ascontiguousarray(a)).to(dev, t)  # noqa: E731
    n = len(d["ts"])
    assert np.bincount(d["terminal"]).max() > 4 * 1024
    ts, term, fr = T(d["ts"], torch.int64), T(d["terminal"], torch.int32), T(d["fraud"], torch.uint8)
    tperm, tseg, tgts, _ = ops.rekey_payload(term, 8, ts, flag=fr)
    ref = ops.terminal_windows_grouped(tgts, tseg, rows=tperm).cpu().numpy()   # by input row
    m = d["terminal"] == 3
    f = oracle.featurize_arrays(d["ts"][m], d["customer"][m], d["terminal"][m], d["amount"][m], d["fraud"][m])
    w = ref[m]
    for j, win in enumerate((1, 7, 30)):
        nb, frc = (w[:, j] & 0xFFFFFFFF).astype(np.int64), w[:, j] >> 32
        np.testing.assert_array_equal(nb, f[f"TERMINAL_ID_NB_TX_{win}DAY_WINDOW"])
        risk = np.where(nb > 0, frc / np.maximum(nb, 1), 0.0)
        np.testing.assert_array_equal(risk, f[f"TERMINAL_ID_RISK_{win}DAY_WINDOW"])
    order = np.argsort(d["customer"] % parts, kind="stable")
    rts, rterm, rfr = T(d["ts"][order], torch.int64), T(d["terminal"][order], torch.int32), \
        T(d["fraud"][order], torch.uint8)
    # the owner side's path: payload re-key (fraud in bit 31 of the perm), grouped runs
    perm, seg, gts, _ = ops.rekey_payload(rterm, 8, rts, flag=rfr)
    got = ops.terminal_windows_grouped(gts, seg, rows=perm, runs=True).cpu().numpy()
    np.testing.assert_array_equal(got, ref[order])
    assert n > 0
