"""Config 5 fed from the wire format: Debezium CDC micro-batches decoded,
deduplicated and compacted on the device, straight into the incremental stream state and the
forest (StreamScorer.score_cdc) -- no host DataFrame in the chain.

  * the record the reference notebook printed (local_dev_notebooks/kafka_s3_sink_transactions.ipynb:318:
    {0, 1736940739000000, 3, 2, LxI=} -> tx 0, 2025-01-15 11:32:19, customer 3, terminal 2,
    120.50; pyspark/scripts/kafka_s3_sink_transactions.py:64-71, :167) scores exactly as the
    decoded row does;
  * a synthetic history streamed as CDC micro-batches with stale duplicate updates (older
    Kafka timestamp, another amount: ROW_NUMBER() ... = 1 at :180 must drop them) gives, batch
    by batch, the probabilities of StreamScorer.score on the true rows, and the kept rows are
    exactly the true records.
"""
import base64
import os
import sys

import numpy as np
import pytest
import torch

from fdx import ops, synth
from fdx.streaming import StreamScorer

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench_stream import cdc_encode  # noqa: E402


def _forest():
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arrays = {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
              for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}
    return ops.Forest(arrays, 15, z["mean"], z["scale"])


def _dev_cdc(r, dev):
    T = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    return (T(r["tx_id"], torch.int64), T(r["customer"], torch.int64), T(r["terminal"], torch.int64),
            T(r["blob"] if len(r["blob"]) else np.zeros(1, np.uint8), torch.uint8), T(r["offsets"], torch.int64),
            T(r["us"], torch.int64), T(r["kts"], torch.int64))


def test_cdc_chain_notebook_record(dev):
    f = _forest()
    a = StreamScorer(f, 10, 10, max_batch=16)
    wire = dict(tx_id=np.array([0]), customer=np.array([3]), terminal=np.array([2]),
                blob=np.frombuffer(base64.b64decode("LxI="), np.uint8).copy(), offsets=np.array([0, 2]),
                us=np.array([1736940739000000]), kts=np.array([1739250197803]))
    p, rows = a.score_cdc(*_dev_cdc(wire, dev))
    assert rows.cpu().tolist() == [0]
    b = StreamScorer(f, 10, 10, max_batch=16)
    ts = int(np.datetime64("2025-01-15T11:32:19", "ns").astype(np.int64))
    T = lambda v, dt: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    q = b.score(T([ts], torch.int64), T([3], torch.int32), T([120.50], torch.float64), T([2], torch.int32),
                T([0], torch.uint8))
    assert torch.equal(p, q)
    assert a.state.check() is None and b.state.check() is None


def test_cdc_chain_stream_with_stale_updates(dev):
    f = _forest()
    d = synth.generate(800, 1500, 45, seed=77)
    n = len(d["ts"])
    cap = 6000
    a = StreamScorer(f, 800, 1500, max_batch=cap)     # fed the CDC wire columns
    b = StreamScorer(f, 800, 1500, max_batch=cap)     # fed the true rows
    T = lambda x, dt: torch.from_numpy(np.ascontiguousarray(x)).to(dev, dt)  # noqa: E731
    cuts = np.r_[np.arange(0, n, 5000), n]
    kts = np.arange(n, dtype=np.int64) * 10 + 1_739_000_000_000
    for k, (lo, hi) in enumerate(zip(cuts[:-1], cuts[1:])):
        r = cdc_encode(np.arange(lo, hi), d["customer"][lo:hi], d["terminal"][lo:hi], d["amount"][lo:hi],
                       d["ts"][lo:hi], kts[lo:hi], dup_frac=0.05, seed=k)
        assert len(r["tx_id"]) > hi - lo
        p, rows = a.score_cdc(*_dev_cdc(r, dev), fraud=None)
        kept = r["tx_id"][rows.cpu().numpy()]
        np.testing.assert_array_equal(kept, np.arange(lo, hi))      # the true records, batch order
        q = b.score(T(d["ts"][lo:hi], torch.int64), T(d["customer"][lo:hi], torch.int32),
                    T(d["amount"][lo:hi], torch.float64), T(d["terminal"][lo:hi], torch.int32),
                    torch.zeros(hi - lo, dtype=torch.uint8, device=dev))
        assert torch.equal(p, q), k
    a.finish()
    b.finish()
