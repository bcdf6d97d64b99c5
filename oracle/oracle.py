"""CPU oracle for the fdx hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It is the checker, never the thing measured or shipped: the
product path (``fdx`` package -> ``libfdx.so`` -> HIP kernels) must not import it and
raises if its HIP extension is missing.

Contents
  * ``liboracle.so`` (``fdx_oracle.c``): pandas roll_sum / variable-window-bounds and
    sklearn forest traversal restated in C (see that file's header for the exact
    third-party algorithms and versions, and the reference call sites).
  * numpy restatements of ``is_weekend`` / ``is_night``
    (fraud_detection_model/feature_transformation.ipynb:246-253, :294-301) and of the
    Spark SQL flags (pyspark/scripts/fraud_detection.py:103-104).
  * ``featurize_table``: the notebook driver (feature_transformation.ipynb:1092-1093,
    :2435-2436) over a whole transaction table.

Parity is pinned by tests/golden/ (vectors produced by running the reference's own
notebook functions, script: oracle/gen_golden.py) and by the notebook-printed known
answer rows (tests/golden/notebook_kat.json).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

NS_PER_DAY = 86_400 * 1_000_000_000
CUSTOMER_COLS = [f"CUSTOMER_ID_{k}_{w}DAY_WINDOW" for w in (1, 7, 30) for k in ("NB_TX", "AVG_AMOUNT")]
TERMINAL_COLS = [f"TERMINAL_ID_{k}_{w}DAY_WINDOW" for w in (1, 7, 30) for k in ("NB_TX", "RISK")]
INPUT_FEATURES = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + CUSTOMER_COLS + TERMINAL_COLS


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        L.oracle_customer_windows.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_int32, P, P]
        L.oracle_terminal_windows.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int64, P,
                                              ctypes.c_int32, P, P]
        L.oracle_forest_predict.argtypes = [P, ctypes.c_int64, ctypes.c_int32, P, P, ctypes.c_int32,
                                            P, P, P, P, P, P, P, P, P]
        for f in (L.oracle_customer_windows, L.oracle_terminal_windows, L.oracle_forest_predict):
            f.restype = ctypes.c_int
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


# ----------------------------------------------------------------------------- flags
def weekend_flag(ts_ns: np.ndarray) -> np.ndarray:
    """Timestamp.weekday() >= 5 (feature_transformation.ipynb:246-253). 1970-01-01 = Thursday."""
    days = np.floor_divide(ts_ns.astype(np.int64), NS_PER_DAY)
    return (((days + 3) % 7) >= 5).astype(np.int64)


def night_flag(ts_ns: np.ndarray) -> np.ndarray:
    """Timestamp.hour <= 6 (feature_transformation.ipynb:294-301)."""
    sod = np.mod(ts_ns.astype(np.int64), NS_PER_DAY)
    return ((sod // (3600 * 1_000_000_000)) <= 6).astype(np.int64)


def spark_weekend_flag(ts_ns):
    """Spark ``dayofweek(ts) >= 5`` (1=Sunday..7=Saturday) -> Thu/Fri/Sat (fraud_detection.py:103)."""
    days = np.floor_divide(ts_ns.astype(np.int64), NS_PER_DAY)
    dow = ((days + 4) % 7) + 1
    return (dow >= 5).astype(np.int64)


def spark_night_flag(ts_ns):
    """Spark ``hour(ts) >= 20`` with a UTC session time zone (fraud_detection.py:104)."""
    sod = np.mod(ts_ns.astype(np.int64), NS_PER_DAY)
    return ((sod // (3600 * 1_000_000_000)) >= 20).astype(np.int64)


# --------------------------------------------------------------------------- windows
def group_order(keys: np.ndarray, ts_ns: np.ndarray):
    """Stable order by (key, ts, input position) + CSR offsets over the sorted keys."""
    order = np.lexsort((np.arange(len(keys)), ts_ns, keys))
    sk = keys[order]
    if len(sk):
        starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
    else:
        starts = np.zeros(0, dtype=np.int64)
    seg_off = np.r_[starts, len(sk)].astype(np.int64)
    return order, seg_off


def customer_windows(ts_ns, amount, seg_off, windows_days=(1, 7, 30)):
    """Rows already grouped + time-ordered. Returns (nb[W][n], avg[W][n]) float64."""
    ts_ns = np.ascontiguousarray(ts_ns, dtype=np.int64)
    amount = np.ascontiguousarray(amount, dtype=np.float64)
    seg_off = np.ascontiguousarray(seg_off, dtype=np.int64)
    win = np.asarray([w * NS_PER_DAY for w in windows_days], dtype=np.int64)
    n = len(ts_ns)
    nb = np.zeros((len(win), n)); avg = np.zeros((len(win), n))
    rc = lib().oracle_customer_windows(_p(ts_ns), _p(amount), _p(seg_off), len(seg_off) - 1,
                                       _p(win), len(win), _p(nb), _p(avg))
    assert rc == 0
    return nb, avg


def terminal_windows(ts_ns, fraud, seg_off, delay_days=7, windows_days=(1, 7, 30)):
    ts_ns = np.ascontiguousarray(ts_ns, dtype=np.int64)
    fraud = np.ascontiguousarray(fraud, dtype=np.float64)
    seg_off = np.ascontiguousarray(seg_off, dtype=np.int64)
    win = np.asarray([w * NS_PER_DAY for w in windows_days], dtype=np.int64)
    n = len(ts_ns)
    nb = np.zeros((len(win), n)); risk = np.zeros((len(win), n))
    rc = lib().oracle_terminal_windows(_p(ts_ns), _p(fraud), _p(seg_off), len(seg_off) - 1,
                                       delay_days * NS_PER_DAY, _p(win), len(win), _p(nb), _p(risk))
    assert rc == 0
    return nb, risk


def featurize_arrays(ts_ns, customer_id, terminal_id, amount, fraud,
                     windows_days=(1, 7, 30), delay_days=7):
    """All 14 derived features for a table in its input row order (dict of float64/int64)."""
    ts_ns = np.asarray(ts_ns, dtype=np.int64)
    n = len(ts_ns)
    out = {"TX_DURING_WEEKEND": weekend_flag(ts_ns), "TX_DURING_NIGHT": night_flag(ts_ns)}
    order, seg = group_order(np.asarray(customer_id), ts_ns)
    nb, avg = customer_windows(ts_ns[order], np.asarray(amount, np.float64)[order], seg, windows_days)
    for k, w in enumerate(windows_days):
        a = np.empty(n); a[order] = nb[k]; out[f"CUSTOMER_ID_NB_TX_{w}DAY_WINDOW"] = a
        b = np.empty(n); b[order] = avg[k]; out[f"CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW"] = b
    order, seg = group_order(np.asarray(terminal_id), ts_ns)
    nb, risk = terminal_windows(ts_ns[order], np.asarray(fraud, np.float64)[order], seg,
                                delay_days, windows_days)
    for k, w in enumerate(windows_days):
        a = np.empty(n); a[order] = nb[k]; out[f"TERMINAL_ID_NB_TX_{w}DAY_WINDOW"] = a
        b = np.empty(n); b[order] = risk[k]; out[f"TERMINAL_ID_RISK_{w}DAY_WINDOW"] = b
    return out


def featurize_table(df):
    """Notebook driver over a pandas frame: returns a copy with the 14 columns added,
    sorted by TX_DATETIME (stable on input order), index reset (:1093, :2436)."""
    import pandas as pd
    ts = df["TX_DATETIME"].values.astype("datetime64[ns]").astype(np.int64)
    feats = featurize_arrays(ts, df["CUSTOMER_ID"].values.astype(np.int64),
                             df["TERMINAL_ID"].values.astype(np.int64),
                             df["TX_AMOUNT"].values, df["TX_FRAUD"].values)
    out = df.copy()
    for k, v in feats.items():
        out[k] = v
    out = out.iloc[np.argsort(ts, kind="stable")].reset_index(drop=True)
    return out


# ---------------------------------------------------------------------------- forest
def forest_arrays(model):
    """Concatenate sklearn tree arrays (estimators_ for forests, the tree itself otherwise)."""
    ests = getattr(model, "estimators_", None) or [model]
    left, right, feat, thr, ml, val, off = [], [], [], [], [], [], [0]
    for e in ests:
        t = e.tree_
        left.append(t.children_left.astype(np.int64)); right.append(t.children_right.astype(np.int64))
        feat.append(t.feature.astype(np.int64)); thr.append(t.threshold.astype(np.float64))
        ml.append(np.asarray(t.missing_go_to_left, dtype=np.uint8))
        val.append(t.value[:, 0, 1].astype(np.float64))
        off.append(off[-1] + t.node_count)
    return dict(left=np.concatenate(left), right=np.concatenate(right), feature=np.concatenate(feat),
                threshold=np.concatenate(thr), missing_left=np.concatenate(ml),
                value1=np.concatenate(val), node_offsets=np.asarray(off, np.int64))


def forest_predict(X, arrays, mean=None, scale=None, want_leaves=False):
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, nf = X.shape
    nt = len(arrays["node_offsets"]) - 1
    proba = np.zeros(n)
    leaves = np.zeros((n, nt), np.int32) if want_leaves else None
    m = None if mean is None else np.ascontiguousarray(mean, np.float64)
    s = None if scale is None else np.ascontiguousarray(scale, np.float64)
    a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
    rc = lib().oracle_forest_predict(_p(X), n, nf, _p(m), _p(s), nt, _p(a["node_offsets"]), _p(a["left"]),
                                     _p(a["right"]), _p(a["feature"]), _p(a["threshold"]),
                                     _p(a["missing_left"]), _p(a["value1"]), _p(proba), _p(leaves))
    assert rc == 0
    return (proba, leaves) if want_leaves else proba
