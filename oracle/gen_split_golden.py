"""Golden vectors for SURVEY §8(f) row f-4 (TEST INFRASTRUCTURE ONLY; build container only):
runs the reference's OWN get_train_test_set (shared_functions.py:133-188) and
card_precision_top_k (shared_functions.py:352-411), exec'd from shared_functions.py by
oracle/refexec.py, on the committed golden frame tests/golden/tiny_a.npz, and writes the
results to tests/golden/split_cpk.npz:

  train_ids / test_ids          TRANSACTION_IDs of get_train_test_set(df, start, 7, 7, 7)
  for start in three dates: train_ids_<k>, test_ids_<k>, start_ns_<k>
  cpk inputs: pred (float64, distinct values: no tie at any top-k boundary), day, customer,
  fraud; outputs nb_comp_<k>, cp_<k>, mean_<k> for top_k in (5, 20) with and without the
  removal of detected cards.

usage: python oracle/gen_split_golden.py
"""
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)


def frame():
    z = np.load(os.path.join(ROOT, "tests", "golden", "tiny_a.npz"))
    o = np.argsort(z["TRANSACTION_ID"], kind="stable")
    df = pd.DataFrame({k: z[k][o] for k in z.files})
    df["TX_DATETIME"] = df["TX_DATETIME"].astype("datetime64[ns]")
    start = np.datetime64("2024-06-01T00:00:00", "ns")
    df["TX_TIME_DAYS"] = ((df["TX_DATETIME"].values - start) // np.timedelta64(1, "D")).astype(np.int64)
    return df.reset_index(drop=True)


def main():
    import refexec

    ns = refexec.load_namespace()
    for fname in ("get_train_test_set", "card_precision_top_k_day", "card_precision_top_k"):
        exec(compile(refexec._shared_function_src(fname), f"<ref:shared_functions.py:{fname}>", "exec"), ns)
    df = frame()
    out = {}
    starts = [pd.Timestamp("2024-06-08"), pd.Timestamp("2024-06-20"), pd.Timestamp("2024-07-03")]
    for k, st in enumerate(starts):
        tr, te = ns["get_train_test_set"](df, st, delta_train=7, delta_delay=7, delta_test=7)
        out[f"train_ids_{k}"] = tr.TRANSACTION_ID.values.astype(np.int64)
        out[f"test_ids_{k}"] = te.TRANSACTION_ID.values.astype(np.int64)
        out[f"start_ns_{k}"] = np.int64(st.value)
    rng = np.random.default_rng(5)
    pred = rng.random(len(df))
    pred[df.TX_FRAUD.values == 1] += 0.3                      # a useful detector
    out["pred"] = pred
    pdf = df[["TX_TIME_DAYS", "CUSTOMER_ID", "TX_FRAUD"]].copy()
    pdf["predictions"] = pred
    k = 0
    for top_k in (5, 20):
        for rem in (True, False):
            nb, cp, mean = ns["card_precision_top_k"](pdf, top_k, remove_detected_compromised_cards=rem)
            out[f"cpk_topk_{k}"] = np.int64(top_k)
            out[f"cpk_remove_{k}"] = np.int64(rem)
            out[f"nb_comp_{k}"] = np.asarray(nb, np.int64)
            out[f"cp_{k}"] = np.asarray(cp, np.float64)
            out[f"mean_{k}"] = np.float64(mean)
            k += 1
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "split_cpk.npz"), **out)
    print({kk: (v.shape if hasattr(v, "shape") else v) for kk, v in out.items()})


if __name__ == "__main__":
    main()
