"""the delay-aware train/test split and Card-Precision@k, so that
model-quality parity (model_training.ipynb:2329-2341: AUC ROC, AP, CP@100) runs on the GPU
outputs.  Same names, arguments and return shapes as the reference:

  get_train_test_set(transactions_df, start_date_training, delta_train=7, delta_delay=7,
                     delta_test=7, sampling_ratio=1.0, random_state=0)
                                                        shared_functions.py:133-188
  card_precision_top_k(predictions_df, top_k, remove_detected_compromised_cards=True)
                                                        shared_functions.py:384-411
The row selection (split masks, per-day per-card maxima, top-k) runs in libfdx.so
(csrc/fdx_aux.hip).  sampling_ratio < 1 subsamples the train set with pandas' own
DataFrame.sample (the reference's RNG), on the host.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pandas as pd
import torch

from . import _lib, ops
from ._lib import check
from .features import _dense_keys, _to_dev, _ts_ns


def get_train_test_set(transactions_df: pd.DataFrame, start_date_training, delta_train=7, delta_delay=7,
                       delta_test=7, sampling_ratio=1.0, random_state=0):
    dev = ops.require_gpu()
    df = transactions_df
    n = len(df)
    ts = _to_dev(_ts_ns(df["TX_DATETIME"].values), torch.int64, dev)
    day = _to_dev(df["TX_TIME_DAYS"].values.astype(np.int32), torch.int32, dev)
    cust, n_cust = _dense_keys(df["CUSTOMER_ID"].values, dev)
    fraud = _to_dev((df["TX_FRAUD"].values != 0).astype(np.uint8), torch.uint8, dev)
    t_lo = int(pd.Timestamp(start_date_training).value)
    t_hi = t_lo + int(delta_train) * ops.NS_PER_DAY
    train = torch.empty(n, dtype=torch.uint8, device=dev)
    test = torch.empty(n, dtype=torch.uint8, device=dev)
    ws = ops.workspace(n_cust * 5 + 64, dev)
    dmin = ctypes.c_int32(0)
    check(_lib.load().fdx_train_test_split(ops._ptr(ts), ops._ptr(day), ops._ptr(cust), ops._ptr(fraud), n, n_cust,
                                           t_lo, t_hi, int(delta_train), int(delta_delay), int(delta_test),
                                           ops._ptr(train), ops._ptr(test), ops._ptr(ws), ws.numel(),
                                           ctypes.byref(dmin), ops._s()), "fdx_train_test_split")
    train_df = df[train.cpu().numpy().astype(bool)]
    test_df = df[test.cpu().numpy().astype(bool)]
    if sampling_ratio < 1:
        train_df_frauds = train_df[train_df.TX_FRAUD == 1].sample(frac=sampling_ratio, random_state=random_state)
        train_df_genuine = train_df[train_df.TX_FRAUD == 0].sample(frac=sampling_ratio, random_state=random_state)
        train_df = pd.concat([train_df_frauds, train_df_genuine])
    return train_df.sort_values("TRANSACTION_ID"), test_df.sort_values("TRANSACTION_ID")


def card_precision_top_k(predictions_df: pd.DataFrame, top_k: int, remove_detected_compromised_cards=True):
    """-> (nb_compromised_cards_per_day, card_precision_top_k_per_day_list, mean)."""
    dev = ops.require_gpu()
    df = predictions_df
    days = np.sort(df["TX_TIME_DAYS"].unique()).astype(np.int32)
    pred = df["predictions"].values.astype(np.float64)
    if len(pred) and (pred.min() < 0 or np.isnan(pred).any()):
        raise _lib.FdxUnsupported("predictions must be >= 0 and not NaN")
    day = _to_dev(df["TX_TIME_DAYS"].values.astype(np.int32), torch.int32, dev)
    cust, n_cust = _dense_keys(df["CUSTOMER_ID"].values, dev)
    fraud = _to_dev((df["TX_FRAUD"].values != 0).astype(np.uint8), torch.uint8, dev)
    L = _lib.load()
    ws = ops.workspace(L.fdx_card_precision_workspace_size(n_cust), dev)
    nb = np.zeros(len(days), np.int32)
    cp = np.zeros(len(days), np.float64)
    check(L.fdx_card_precision_top_k(ops._ptr(day), ops._ptr(cust), ops._ptr(_to_dev(pred, torch.float64, dev)),
                                     ops._ptr(fraud), len(df), n_cust, days.ctypes.data, len(days), int(top_k),
                                     int(bool(remove_detected_compromised_cards)), nb.ctypes.data, cp.ctypes.data,
                                     ops._ptr(ws), ws.numel(), ops._s()), "fdx_card_precision_top_k")
    return nb.tolist(), cp.tolist(), float(np.array(cp).mean())
