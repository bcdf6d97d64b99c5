"""the batch -> streaming hand-off either side of the hot path.

f-1 feature snapshots (the tables the Spark scoring job LEFT JOINs, fraud_detection.py:118-122),
  from a frame (below) or straight from the featurized table the scoring step writes
  (latest_terminal_features_from_table, customer_features_on_from_table: fdx_table_select):
  latest_terminal_features(df)     feature_transformation.ipynb:2914-2918
      df.loc[df.groupby('TERMINAL_ID').TX_DATETIME.idxmax()].filter(regex='TERMINAL_ID|TERMINAL_ID_RISK')
  customer_features_on(df, date)   :3461, :3606-3635, :4182
      lower-cased columns, filter(regex='customer_id|tx_datetime'), rows of `date`,
      dt = date, drop tx_datetime, drop_duplicates(subset=['customer_id'])  (keep='first')
f-2 Debezium CDC micro-batch decode (pyspark/scripts/kafka_s3_sink_transactions.py)
  decode_cdc_batch(...)            :64-71 (tx_amount), :167 (tx_datetime), :180 (latest per tx_id)

Device tensors in, device tensors / pandas frames out; the row selection (segmented arg-max,
first-in-range, byte decode, dedup) runs in libfdx.so (csrc/fdx_aux.hip).
"""
from __future__ import annotations

import datetime

import numpy as np
import pandas as pd
import torch

from . import _lib, ops
from ._lib import check
from .features import _dense_keys, _to_dev, _ts_ns

NS_PER_DAY = ops.NS_PER_DAY


# ------------------------------------------------------------------------------ device layer
def segment_latest(ts_ns: torch.Tensor, perm: torch.Tensor, seg_off: torch.Tensor, stream=None) -> torch.Tensor:
    """Per segment of a stable grouping: the row holding the segment's max ts (first such row
    in frame order), -1 for an empty segment."""
    n_seg = seg_off.numel() - 1
    out = torch.empty(max(n_seg, 0), dtype=torch.int32, device=ts_ns.device)
    check(_lib.load().fdx_segment_latest(ops._ptr(ts_ns), ops._ptr(perm), ops._ptr(seg_off), n_seg, ops._ptr(out),
                                         ops._s(stream)), "fdx_segment_latest")
    return out


def segment_first_in_range(ts_ns, perm, seg_off, t_lo: int, t_hi: int, stream=None) -> torch.Tensor:
    """Per segment: the first row (frame order) with t_lo <= ts < t_hi, -1 if none."""
    n_seg = seg_off.numel() - 1
    out = torch.empty(max(n_seg, 0), dtype=torch.int32, device=ts_ns.device)
    check(_lib.load().fdx_segment_first_in_range(ops._ptr(ts_ns), ops._ptr(perm), ops._ptr(seg_off), n_seg,
                                                 int(t_lo), int(t_hi), ops._ptr(out), ops._s(stream)),
          "fdx_segment_first_in_range")
    return out


def cdc_decode(amount_bytes: torch.Tensor | None, offsets: torch.Tensor | None, tx_datetime_us: torch.Tensor | None,
               stream=None):
    """-> (unscaled int64 cents | None, amount float64 | None, ts_ns int64 | None)."""
    dev = (amount_bytes if amount_bytes is not None else tx_datetime_us).device
    n = offsets.numel() - 1 if offsets is not None else tx_datetime_us.numel()
    uns = amt = tsn = None
    if amount_bytes is not None:
        ops._dev(amount_bytes, torch.uint8, "amount_bytes"); ops._dev(offsets, torch.int64, "offsets")
        uns = torch.empty(n, dtype=torch.int64, device=dev)
        amt = torch.empty(n, dtype=torch.float64, device=dev)
    if tx_datetime_us is not None:
        ops._dev(tx_datetime_us, torch.int64, "tx_datetime_us")
        if tx_datetime_us.numel() != n:
            raise _lib.FdxError("one tx_datetime per record")
        tsn = torch.empty(n, dtype=torch.int64, device=dev)
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    check(_lib.load().fdx_cdc_decode(ops._ptr(amount_bytes), ops._ptr(offsets), ops._ptr(tx_datetime_us), n,
                                     ops._ptr(uns), ops._ptr(amt), ops._ptr(tsn), ops._ptr(bad), ops._s(stream)),
          "fdx_cdc_decode")
    if int(bad.item()):
        raise _lib.FdxUnsupported("a tx_amount field has 0 or more than 8 bytes")
    return uns, amt, tsn


def dedup_latest(key: torch.Tensor, kafka_ts: torch.Tensor, bad: torch.Tensor | None = None, stream=None):
    """uint8 keep mask: the record with the largest Kafka timestamp per key (ties: last).
    bad (int32 device scalar, optional): set to 1 if a key is -1 (the hash table's empty key)."""
    ops._dev(key, torch.int64, "key"); ops._dev(kafka_ts, torch.int64, "kafka_ts")
    n = key.numel()
    keep = torch.empty(n, dtype=torch.uint8, device=key.device)
    L = _lib.load()
    ws = ops.workspace(L.fdx_dedup_latest_workspace_size(n), key.device)
    own = bad is None
    if own:
        bad = torch.zeros(1, dtype=torch.int32, device=key.device)
    check(L.fdx_dedup_latest(ops._ptr(key), ops._ptr(kafka_ts), n, ops._ptr(keep), ops._ptr(bad), ops._ptr(ws),
                             ws.numel(), ops._s(stream)), "fdx_dedup_latest")
    if own and n and int(bad.item()):
        raise _lib.FdxUnsupported("tx_id -1 is reserved (the dedup table's empty key)")
    return keep


def table_select(rows, n_slots: int, ts_ns: torch.Tensor, key: torch.Tensor, n_keys: int, mode: int,
                 t_lo: int = 0, t_hi: int = 0, stream=None) -> torch.Tensor:
    """Per key: the slot of the featurized table (ops.FeatureTable, slot order) holding the row
    fdx_table_select picks (FDX_SELECT_LATEST / FDX_SELECT_FIRST_IN_RANGE), -1 if none.
    ts_ns / key: by input row (time order)."""
    if not isinstance(rows, ops.FeatureTable):
        raise TypeError("table_select reads an ops.FeatureTable (slot order)")
    ops._dev(ts_ns, torch.int64, "ts_ns"); ops._dev(key, torch.int32, "key")
    n_slots = int(n_slots)
    if not 0 <= n_slots <= rows.cap:
        raise ValueError(f"n_slots {n_slots} outside the table's [0, {rows.cap}] slots")
    if ts_ns.numel() != key.numel():
        raise ValueError(f"ts_ns has {ts_ns.numel()} rows, key {key.numel()}")
    out = torch.empty(max(int(n_keys), 0), dtype=torch.int32, device=ts_ns.device)
    L = _lib.load()
    ws = ops.workspace(L.fdx_table_select_workspace_size(int(n_keys)), ts_ns.device)
    row = rows.columns(n_slots)["row"]
    # the kernel reads ts_ns / key at every slot's row: a table from another frame would read out of
    # bounds (one host read; snapshot export, not the scoring step)
    if n_slots and int(row.max()) >= ts_ns.numel():
        raise ValueError("the table's rows index past ts_ns / key: a table written for another frame?")
    check(L.fdx_table_select(ops._ptr(row), int(n_slots), ops._ptr(ts_ns), ops._ptr(key), int(n_keys), int(mode),
                             int(t_lo), int(t_hi), ops._ptr(out), ops._ptr(ws), ws.numel(), ops._s(stream)),
          "fdx_table_select")
    return out


def _windows_label(w):
    return f"{w}DAY_WINDOW"


def _original_ids(dense: np.ndarray, ids) -> np.ndarray:
    """dense key -> the frame's id (int64, the pandas dtype of the reference's id columns)"""
    return (dense if ids is None else np.asarray(ids)[dense]).astype(np.int64)


def latest_terminal_features_from_table(rows, n_slots: int, ts_ns: torch.Tensor, terminal: torch.Tensor,
                                        n_terminals: int, windows_days=(1, 7, 30), ids=None) -> pd.DataFrame:
    """feature_transformation.ipynb:2914-2918 on the table the scoring step wrote:
    df.loc[df.groupby('TERMINAL_ID').TX_DATETIME.idxmax()].filter(regex='TERMINAL_ID|TERMINAL_ID_RISK')
    -- index = the chosen input rows, rows in terminal order, the reference table's column
    order and dtypes (counts as float64, as pandas' rolling count; ids int64).  terminal holds
    the dense keys the step ran on; ids (optional): dense key -> the frame's TERMINAL_ID, when
    the frame's ids are not already 0..n-1."""
    slots = table_select(rows, n_slots, ts_ns, terminal, n_terminals, _lib.FDX_SELECT_LATEST)
    keep = slots >= 0
    s = slots[keep].long()
    col = rows.columns(n_slots)
    r = col["row"][s].long()
    out = {"TERMINAL_ID": _original_ids(terminal[r].cpu().numpy(), ids)}
    nb, rk = col["term_nb"][:, s].cpu().numpy(), col["term_risk"][:, s].cpu().numpy()
    for j, w in enumerate(windows_days):
        out[f"TERMINAL_ID_NB_TX_{_windows_label(w)}"] = nb[j].astype(np.float64)
        out[f"TERMINAL_ID_RISK_{_windows_label(w)}"] = rk[j]
    return pd.DataFrame(out, index=pd.Index(r.cpu().numpy()))


def customer_features_on_from_table(rows, n_slots: int, ts_ns: torch.Tensor, customer: torch.Tensor,
                                    n_customers: int, date: datetime.date, windows_days=(1, 7, 30),
                                    ids=None) -> pd.DataFrame:
    """feature_transformation.ipynb:3606-3635 on the table the scoring step wrote: each
    customer's first transaction of `date` with its lower-cased customer columns and dt = date,
    rows in frame (input) order, index = those input rows.  ids (optional): dense key -> the
    frame's CUSTOMER_ID (customer_id is int64 either way)."""
    lo = int(np.datetime64(date, "ns").astype(np.int64))
    slots = table_select(rows, n_slots, ts_ns, customer, n_customers, _lib.FDX_SELECT_FIRST_IN_RANGE, lo,
                         lo + NS_PER_DAY)
    s = slots[slots >= 0].long()
    col = rows.columns(n_slots)
    r = col["row"][s].long()
    o = torch.argsort(r)  # drop_duplicates keeps frame order
    s, r = s[o], r[o]
    out = {"customer_id": _original_ids(customer[r].cpu().numpy(), ids)}
    nb, av = col["cust_nb"][:, s].cpu().numpy(), col["cust_avg"][:, s].cpu().numpy()
    for j, w in enumerate(windows_days):
        out[f"customer_id_nb_tx_{_windows_label(w).lower()}"] = nb[j].astype(np.float64)
        out[f"customer_id_avg_amount_{_windows_label(w).lower()}"] = av[j]
    f = pd.DataFrame(out, index=pd.Index(r.cpu().numpy()))
    f["dt"] = date
    return f


# ------------------------------------------------------------------------------ pandas layer
def _grouping(df: pd.DataFrame, key_col: str, dev):
    keys_d, n_keys = _dense_keys(df[key_col].values, dev)
    perm, seg, _ = ops.rekey(keys_d, n_keys)           # stable: frame order inside a key
    return perm, seg


def latest_terminal_features(transactions_df: pd.DataFrame, key: str = "TERMINAL_ID") -> pd.DataFrame:
    """feature_transformation.ipynb:2914-2918: the latest row of every terminal (first of the
    tied maxima of TX_DATETIME, as idxmax), terminal columns only, rows in key order."""
    dev = ops.require_gpu()
    df = transactions_df
    ts_d = _to_dev(_ts_ns(df["TX_DATETIME"].values), torch.int64, dev)
    perm, seg = _grouping(df, key, dev)
    rows = segment_latest(ts_d, perm, seg).cpu().numpy()
    rows = rows[rows >= 0]                              # dense-id gaps (absent keys)
    out = df.iloc[rows]
    return out.filter(regex=f"{key}|{key}_RISK")


def customer_features_on(transactions_df: pd.DataFrame, date: datetime.date) -> pd.DataFrame:
    """feature_transformation.ipynb:3461, :3606-3635, :4182: each customer's first
    transaction of `date` (frame order) with its customer features, dt = date."""
    dev = ops.require_gpu()
    df = transactions_df.copy()
    df.columns = map(str.lower, df.columns)
    df = df.filter(regex="customer_id|tx_datetime")
    ts_d = _to_dev(_ts_ns(df["tx_datetime"].values), torch.int64, dev)
    perm, seg = _grouping(df, "customer_id", dev)
    lo = int(np.datetime64(date, "ns").astype(np.int64))
    rows = segment_first_in_range(ts_d, perm, seg, lo, lo + NS_PER_DAY).cpu().numpy()
    rows = np.sort(rows[rows >= 0])                     # drop_duplicates keeps frame order
    out = df.iloc[rows].copy()
    out["dt"] = out["tx_datetime"].dt.date
    return out.drop(columns=["tx_datetime"])


def decode_cdc_batch(tx_id, customer_id, terminal_id, tx_amount_bytes, tx_datetime_us, kafka_timestamp) -> pd.DataFrame:
    """kafka_s3_sink_transactions.py:160-186 on one micro-batch: decode tx_amount
    (DECIMAL(10,2) bytes) and tx_datetime (us -> whole seconds), keep the latest record per
    tx_id by Kafka timestamp.  Returns the kept rows in batch order with tx_amount as
    float64 (and tx_amount_cents, the exact unscaled value)."""
    dev = ops.require_gpu()
    tx_id = np.asarray(tx_id, np.int64)
    n = len(tx_id)
    lens = np.fromiter((len(b) for b in tx_amount_bytes), np.int64, n)
    offsets = np.r_[0, np.cumsum(lens)].astype(np.int64)
    blob = np.frombuffer(b"".join(bytes(b) for b in tx_amount_bytes), np.uint8).copy() if n else np.zeros(0, np.uint8)
    uns, amt, tsn = cdc_decode(_to_dev(blob if len(blob) else np.zeros(1, np.uint8), torch.uint8, dev),
                               _to_dev(offsets, torch.int64, dev),
                               _to_dev(np.asarray(tx_datetime_us, np.int64), torch.int64, dev))
    kts = np.asarray(kafka_timestamp).astype("datetime64[ns]").astype(np.int64) \
        if not np.issubdtype(np.asarray(kafka_timestamp).dtype, np.integer) else np.asarray(kafka_timestamp, np.int64)
    keep = dedup_latest(_to_dev(tx_id, torch.int64, dev), _to_dev(kts, torch.int64, dev)).cpu().numpy().astype(bool)
    out = pd.DataFrame({
        "tx_id": tx_id, "tx_datetime": tsn.cpu().numpy().astype("datetime64[ns]"),
        "customer_id": np.asarray(customer_id), "terminal_id": np.asarray(terminal_id),
        "tx_amount": amt.cpu().numpy(), "tx_amount_cents": uns.cpu().numpy()})
    return out[keep].reset_index(drop=True)
