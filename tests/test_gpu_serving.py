"""SURVEY.md §8(f) rows f-1 (feature snapshots) and f-2 (Debezium CDC decode + dedup) on the
GPU against the reference's own expressions (pandas, the reference's library, run here on
the same frames) and the CDC record the reference notebook printed.

  f-1  feature_transformation.ipynb:2914-2918, :3461, :3606-3635, :4182
  f-2  pyspark/scripts/kafka_s3_sink_transactions.py:64-71, :167, :180;
       local_dev_notebooks/kafka_s3_sink_transactions.ipynb:318 (a decoded record)
"""
import base64
import datetime
from decimal import Decimal

import numpy as np
import pandas as pd
import pytest

from fdx import serving

pytestmark = pytest.mark.gpu


def _frame(golden, name="tiny_a.npz"):
    z = golden(name)
    o = np.argsort(z["TRANSACTION_ID"], kind="stable")
    df = pd.DataFrame({k: z[k][o] for k in z.files})
    df["TX_DATETIME"] = df["TX_DATETIME"].astype("datetime64[ns]")
    return df.reset_index(drop=True)


def test_latest_terminal_features_matches_pandas(dev, golden):
    df = _frame(golden)
    ref = df.loc[df.groupby("TERMINAL_ID").TX_DATETIME.idxmax()].filter(regex="TERMINAL_ID|TERMINAL_ID_RISK")
    got = serving.latest_terminal_features(df)
    pd.testing.assert_frame_equal(got, ref)


def test_latest_ties_take_the_first_row(dev, golden):
    """idxmax returns the first of tied maxima (frame order), also when the frame is not
    time-sorted."""
    df = _frame(golden).sample(frac=1.0, random_state=3).reset_index(drop=True)
    df.loc[df.index[:200], "TX_DATETIME"] = df["TX_DATETIME"].max()   # many ties at the max
    ref = df.loc[df.groupby("TERMINAL_ID").TX_DATETIME.idxmax()].filter(regex="TERMINAL_ID|TERMINAL_ID_RISK")
    pd.testing.assert_frame_equal(serving.latest_terminal_features(df), ref)


@pytest.mark.parametrize("day", [0, 17, 59])
def test_customer_features_on_date_matches_pandas(dev, golden, day):
    df = _frame(golden)
    date = (df["TX_DATETIME"].min() + pd.Timedelta(days=day)).date()
    t = df.copy()
    t.columns = map(str.lower, t.columns)
    cf = t.filter(regex="customer_id|tx_datetime")
    cf = cf[cf.tx_datetime.dt.date == date]
    cf = cf.assign(dt=cf["tx_datetime"].dt.date).drop(columns=["tx_datetime"])
    ref = cf.drop_duplicates(subset=["customer_id"])
    got = serving.customer_features_on(df, date)
    pd.testing.assert_frame_equal(got, ref)


def _decode_ref(b):
    # kafka_s3_sink_transactions.py:64-71
    return Decimal(int.from_bytes(b, byteorder="big", signed=True)) / (10 ** 2)


def test_cdc_decode_notebook_record(dev):
    """{0, 1736940739000000, 3, 2, LxI=} -> tx 0, 2025-01-15 11:32:19, customer 3, terminal 2,
    120.50 (the record printed at local_dev_notebooks/kafka_s3_sink_transactions.ipynb:318)."""
    out = serving.decode_cdc_batch([0], [3], [2], [base64.b64decode("LxI=")], [1736940739000000],
                                   [1739250197803])
    assert out.tx_id.tolist() == [0]
    assert out.tx_datetime[0] == pd.Timestamp("2025-01-15 11:32:19")
    assert out.tx_amount_cents[0] == 12050 and out.tx_amount[0] == 120.50
    assert out.customer_id[0] == 3 and out.terminal_id[0] == 2


def test_cdc_decode_and_dedup_random_batch(dev):
    rng = np.random.default_rng(7)
    n = 5000
    cents = rng.integers(-(10 ** 10) + 1, 10 ** 10, n)
    cents[:50] = rng.integers(-300, 300, 50)                       # short encodings, signs
    raw = []
    for c in cents:
        c = int(c)
        nbytes = max(1, (c.bit_length() + 8) // 8)                 # minimal two's complement, as Kafka Connect
        raw.append(c.to_bytes(nbytes, "big", signed=True))
    us = rng.integers(1_700_000_000_000_000, 1_760_000_000_000_000, n)
    tx_id = rng.integers(0, 1500, n)                               # many updates per tx_id
    kts = rng.integers(0, 40, n)                                   # Kafka timestamps, ties included
    out = serving.decode_cdc_batch(tx_id, rng.integers(0, 99, n), rng.integers(0, 99, n), raw, us, kts)
    # reference: decode every record, then ROW_NUMBER() OVER (PARTITION BY tx_id ORDER BY
    # timestamp DESC) = 1 (ties -> the last in batch order, our documented choice)
    keep = {}
    for i in range(n):
        j = keep.get(int(tx_id[i]))
        if j is None or kts[i] >= kts[j]:
            keep[int(tx_id[i])] = i
    idx = np.sort(np.array(list(keep.values())))
    np.testing.assert_array_equal(out.tx_id.values, tx_id[idx])
    dec = np.array([float(_decode_ref(raw[i])) for i in idx])
    np.testing.assert_array_equal(out.tx_amount.values, dec)
    np.testing.assert_array_equal(out.tx_amount_cents.values, cents[idx])
    secs = np.array([int(us[i] / 1_000_000) for i in idx], np.int64)   # from_unixtime(us / 1e6)
    np.testing.assert_array_equal(out.tx_datetime.values.astype(np.int64), secs * 1_000_000_000)


@pytest.mark.parametrize("n_slots_extra", [0, 700])
def test_table_select_edges(dev, n_slots_extra):
    """fdx_table_select on a hand-made slot table against numpy: tied timestamps (the first
    input row of the tied maxima, as idxmax), keys without rows (-1), padding slots (row -1),
    rows whose key is out of range (ignored), a time range that holds no row, and an empty
    table."""
    import torch

    from fdx import _lib, ops

    rng = np.random.default_rng(11)
    n, n_keys = 5000, 300
    ts = np.sort(rng.integers(0, 40, n)) * 3_600_000_000_000  # hour-floored: many ties
    key = rng.integers(0, n_keys - 10, n).astype(np.int32)   # keys 290..299 never occur
    key[rng.choice(n, 25, replace=False)] = -1                 # out of range: ignored
    key[rng.choice(n, 25, replace=False)] = n_keys + 7
    rows = np.concatenate([rng.permutation(n), -np.ones(n_slots_extra, np.int64)])
    rows = rows[rng.permutation(len(rows))].astype(np.int32)
    m = len(rows)
    tab = ops.FeatureTable(m, dev)
    tab.columns(m)["row"].copy_(torch.from_numpy(rows))
    ts_d = torch.from_numpy(ts).to(dev)
    key_d = torch.from_numpy(key).to(dev)
    slot_of_row = np.empty(n, np.int64)
    live = rows >= 0
    slot_of_row[rows[live]] = np.nonzero(live)[0]

    def want(pick):
        out = -np.ones(n_keys, np.int32)
        for k in range(n_keys):
            r = pick(np.nonzero(key == k)[0])
            if r is not None:
                out[k] = slot_of_row[r]
        return out

    def latest(rs):
        return None if len(rs) == 0 else rs[np.argmax(ts[rs])]  # first of the tied maxima

    got = serving.table_select(tab, m, ts_d, key_d, n_keys, _lib.FDX_SELECT_LATEST).cpu().numpy()
    np.testing.assert_array_equal(got, want(latest))
    for lo, hi in ((5 * 3_600_000_000_000, 9 * 3_600_000_000_000), (10**18, 10**18 + 5), (0, 1)):
        def first(rs, lo=lo, hi=hi):
            rs = rs[(ts[rs] >= lo) & (ts[rs] < hi)]
            return None if len(rs) == 0 else rs.min()

        got = serving.table_select(tab, m, ts_d, key_d, n_keys, _lib.FDX_SELECT_FIRST_IN_RANGE, lo, hi).cpu().numpy()
        np.testing.assert_array_equal(got, want(first), err_msg=f"[{lo}, {hi})")
    empty = serving.table_select(tab, 0, ts_d, key_d, n_keys, _lib.FDX_SELECT_LATEST).cpu().numpy()
    np.testing.assert_array_equal(empty, -np.ones(n_keys, np.int32))
