"""Builds bench_assets/rf_deployed.npz: the model the reference DEPLOYS (build container only).

model_training.ipynb trains its model zoo with fit_model_and_get_predictions (:2209-2223) and
pickles the 'Random forest' entry -- RandomForestClassifier(random_state=0, n_jobs=-1): 100
trees, unlimited depth (:2212) -- as ../data/trained_model.pkl (:2610-2614), which the Spark
job loads and applies to scaler.transform(features) (pyspark/scripts/fraud_detection.py:81-85,
:190-193).  Its published predict_proba time, 0.4766 s for the 66,452-row test set
(:2524-2525, ~139k rows/s), is the reference's only published scoring number.

Reproduced here step by step:
  data      the reference generator (data_generator.ipynb, 245 days, seeds per customer)
            featurized by the reference's own notebook functions (oracle/refexec.py) over
            2024-06-01 .. 2024-12-31 (feature_transformation.ipynb:91-95), then the model
            notebook's load filter TX_DATETIME <= "2024-12-31" (model_training.ipynb:73-96);
  split     get_train_test_set(delta_train=153, delta_delay=30, delta_test=30)
            (model_training.ipynb:248-304): 1,466,282 train rows (:311);
  scaling   scaleData at :823 -- which scales train/test IN PLACE -- and again inside
            fit_model_and_get_predictions(scale=True) (:496), so the forest is fitted on
            twice-scaled features while the served scaler.pkl is the first one (:1256);
  model     RandomForestClassifier(random_state=0, n_jobs=-1).fit (:2212, :500).
Only arrays are saved (no pickle): tree arrays, the served scaler's mean_/scale_, the
raw (unscaled) test rows and sklearn's predict_proba of scaler.transform(test) with n_jobs=1
(tree-order float64 accumulation), i.e. exactly what the Spark UDF computes.
"""
import os
import sys
import time
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

FEATS = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT",
         "CUSTOMER_ID_NB_TX_1DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_1DAY_WINDOW",
         "CUSTOMER_ID_NB_TX_7DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_7DAY_WINDOW",
         "CUSTOMER_ID_NB_TX_30DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_30DAY_WINDOW",
         "TERMINAL_ID_NB_TX_1DAY_WINDOW", "TERMINAL_ID_RISK_1DAY_WINDOW",
         "TERMINAL_ID_NB_TX_7DAY_WINDOW", "TERMINAL_ID_RISK_7DAY_WINDOW",
         "TERMINAL_ID_NB_TX_30DAY_WINDOW", "TERMINAL_ID_RISK_30DAY_WINDOW"]


def main():
    warnings.filterwarnings("ignore")
    import datetime

    import pandas as pd
    import sklearn.ensemble
    import refexec

    ns = refexec.load_namespace()
    cache = "/tmp/fdx_ref_245d.pkl"
    if os.path.exists(cache):
        df = pd.read_pickle(cache)  # our own cache of the reference generator's output
    else:
        c, t, df = ns["generate_dataset"](n_customers=5000, n_terminals=10000, nb_days=245,
                                          start_date="2024-06-01", r=5)
        df = ns["add_frauds"](c, t, df)
        df.to_pickle(cache)
    feat_cache = "/tmp/fdx_ref_214d_feat.pkl"
    if os.path.exists(feat_cache):
        feat = pd.read_pickle(feat_cache)
    else:
        d = df[(df.TX_DATETIME >= "2024-06-01") & (df.TX_DATETIME < "2025-01-01")].copy()
        d = d.sort_values("TRANSACTION_ID").reset_index(drop=True).replace([-1], 0)
        for col in ("CUSTOMER_ID", "TERMINAL_ID", "TX_TIME_SECONDS", "TX_TIME_DAYS"):
            d[col] = d[col].astype(np.int64)
        t0 = time.time()
        feat = refexec.reference_featurize(ns, d)
        print("featurized", feat.shape, round(time.time() - t0, 1), flush=True)
        feat.to_pickle(feat_cache)
    feat = feat[feat.TX_DATETIME <= "2024-12-31"]
    print("loaded", len(feat), "tx", int(feat.TX_FRAUD.sum()), "frauds (notebook: 2041821 / 17188)", flush=True)
    start = datetime.datetime.strptime("2024-06-01", "%Y-%m-%d")
    train, test = ns["get_train_test_set"](feat, start, delta_train=153, delta_delay=30, delta_test=30)
    print("train", len(train), "test", len(test), "(notebook: 1466282 / 66452)", flush=True)
    raw_test = test[FEATS].values.astype(np.float64).copy()
    train, test, scaler = ns["scaleData"](train, test, FEATS)       # :823 (in place)
    train2, test2, _ = ns["scaleData"](train, test, FEATS)          # :496 inside fit_model_and_get_predictions
    rf = sklearn.ensemble.RandomForestClassifier(random_state=0, n_jobs=-1)
    t0 = time.time()
    rf.fit(train2[FEATS], train2["TX_FRAUD"])
    print("trained", round(time.time() - t0, 1), "s", flush=True)
    ests = rf.estimators_
    off = np.cumsum([0] + [e.tree_.node_count for e in ests]).astype(np.int64)
    cat = lambda f: np.concatenate([f(e.tree_) for e in ests])  # noqa: E731
    rf.set_params(n_jobs=1)  # tree-order float64 accumulation (threads add in completion order)
    Z = scaler.transform(pd.DataFrame(raw_test, columns=FEATS))    # the Spark UDF: served scaler, then the model
    t0 = time.time()
    proba = rf.predict_proba(pd.DataFrame(Z, columns=FEATS))
    print("sklearn predict_proba (n_jobs=1)", len(Z), "rows", round(time.time() - t0, 3), "s", flush=True)
    out = os.path.join(HERE, "rf_deployed.npz")
    np.savez_compressed(
        out,
        node_offsets=off,
        right=cat(lambda t: t.children_right).astype(np.int32),
        left=cat(lambda t: t.children_left).astype(np.int32),
        feature=cat(lambda t: t.feature).astype(np.int8),
        threshold=cat(lambda t: t.threshold).astype(np.float64),
        missing_left=cat(lambda t: np.asarray(t.missing_go_to_left)).astype(np.uint8),
        value1=cat(lambda t: t.value[:, 0, 1]).astype(np.float64),
        value0=cat(lambda t: t.value[:, 0, 0]).astype(np.float64),
        mean=scaler.mean_, scale=scaler.scale_,
        test_X=raw_test, test_proba1=proba[:, 1], test_proba0=proba[:, 0],
        test_fraud=test["TX_FRAUD"].values.astype(np.uint8),
    )
    depth = max(e.tree_.max_depth for e in ests)
    print("nodes", off[-1], "max depth", depth, "size", os.path.getsize(out))


if __name__ == "__main__":
    main()
