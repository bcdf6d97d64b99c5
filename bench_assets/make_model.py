"""Builds bench_assets/rf100_d20.npz: the config-3 scoring model (build container only).

BASELINE.json config 3: RandomForestClassifier(n_estimators=100, max_depth=20,
random_state=0) trained on config-1 scaled features.  Config 1 is the handbook-default
dataset, generated here by the reference's own generator (data_generator.ipynb, first 183
days of the 245-day run, which are identical to the 183-day run because the RNG is seeded
per customer) and featurized by the reference's own notebook functions
(feature_transformation.ipynb) through oracle/refexec.py.  Training follows
model_training.ipynb: train window = 153 days from 2024-06-01 (:248-304), scaleData
(shared_functions.py:114-120), fit.  Only the fitted arrays are saved (no pickle).
"""
import os
import sys
import time
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))


def main():
    warnings.filterwarnings("ignore")
    import pandas as pd
    import sklearn.ensemble
    import refexec

    ns = refexec.load_namespace()
    cache = "/tmp/fdx_ref_245d.pkl"
    if os.path.exists(cache):
        df = pd.read_pickle(cache)  # written by oracle/gen_kat.py from the reference generator
    else:
        c, t, df = ns["generate_dataset"](n_customers=5000, n_terminals=10000, nb_days=245,
                                          start_date="2024-06-01", r=5)
        df = ns["add_frauds"](c, t, df)
        df.to_pickle(cache)
    df = df[df.TX_TIME_DAYS.astype(int) < 183].copy()
    df = df.sort_values("TRANSACTION_ID").reset_index(drop=True).replace([-1], 0)
    for col in ("CUSTOMER_ID", "TERMINAL_ID", "TX_TIME_SECONDS", "TX_TIME_DAYS"):
        df[col] = df[col].astype(np.int64)
    t0 = time.time()
    feat = refexec.reference_featurize(ns, df)
    print("featurized", feat.shape, time.time() - t0, flush=True)
    feats = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT",
             "CUSTOMER_ID_NB_TX_1DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_1DAY_WINDOW",
             "CUSTOMER_ID_NB_TX_7DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_7DAY_WINDOW",
             "CUSTOMER_ID_NB_TX_30DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_30DAY_WINDOW",
             "TERMINAL_ID_NB_TX_1DAY_WINDOW", "TERMINAL_ID_RISK_1DAY_WINDOW",
             "TERMINAL_ID_NB_TX_7DAY_WINDOW", "TERMINAL_ID_RISK_7DAY_WINDOW",
             "TERMINAL_ID_NB_TX_30DAY_WINDOW", "TERMINAL_ID_RISK_30DAY_WINDOW"]
    start = pd.Timestamp("2024-06-01")
    train = feat[(feat.TX_DATETIME >= start) & (feat.TX_DATETIME < start + pd.Timedelta(days=153))].copy()
    test = feat[feat.TX_DATETIME >= start + pd.Timedelta(days=153)].copy()
    print("train rows", len(train), "frauds", int(train.TX_FRAUD.sum()), flush=True)
    train, test, scaler = ns["scaleData"](train, test, feats)
    rf = sklearn.ensemble.RandomForestClassifier(n_estimators=100, max_depth=20, random_state=0, n_jobs=8)
    t0 = time.time()
    rf.fit(train[feats], train["TX_FRAUD"])
    print("trained", time.time() - t0, flush=True)
    ests = rf.estimators_
    off = np.cumsum([0] + [e.tree_.node_count for e in ests]).astype(np.int64)
    cat = lambda f: np.concatenate([f(e.tree_) for e in ests])  # noqa: E731
    # a small held-out sample with sklearn's own answers, for the bench's sanity check
    Xs = feat[feats].values[-4096:].astype(np.float64)
    Zs = scaler.transform(pd.DataFrame(Xs, columns=feats))
    rf.set_params(n_jobs=1)  # tree-order float64 accumulation (threads add in completion order)
    np.savez_compressed(
        os.path.join(HERE, "rf100_d20.npz"),
        node_offsets=off,
        right=cat(lambda t: t.children_right).astype(np.int32),
        left=cat(lambda t: t.children_left).astype(np.int32),
        feature=cat(lambda t: t.feature).astype(np.int8),
        threshold=cat(lambda t: t.threshold).astype(np.float64),
        missing_left=cat(lambda t: np.asarray(t.missing_go_to_left)).astype(np.uint8),
        value1=cat(lambda t: t.value[:, 0, 1]).astype(np.float64),
        mean=scaler.mean_, scale=scaler.scale_,
        check_X=Xs, check_proba=rf.predict_proba(pd.DataFrame(Zs, columns=feats))[:, 1],
    )
    print("nodes", off[-1], "size", os.path.getsize(os.path.join(HERE, "rf100_d20.npz")))


if __name__ == "__main__":
    main()
