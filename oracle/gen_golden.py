"""Golden vectors from the reference's own functions.  TEST INFRASTRUCTURE ONLY.

Runs only in the build container (needs /root/reference; exec's the notebook defs through
oracle/refexec.py).  Writes small fixtures to tests/golden/:

  tiny_<name>.npz   inputs (TRANSACTION_ID, TX_DATETIME ns, CUSTOMER_ID, TERMINAL_ID,
                    TX_AMOUNT, TX_FRAUD) + every derived column, as produced by
                    generate_dataset/add_frauds (data_generator.ipynb:1339-1371, :1732-1782)
                    and the notebook driver (feature_transformation.ipynb:278, :319,
                    :1092-1093, :2435-2436), keyed by TRANSACTION_ID.
  ties.npz          same, on a table whose timestamps are floored to the hour so that many
                    (CUSTOMER_ID, TX_DATETIME) ties exist; pandas' per-group quicksort order
                    for tied rows is recovered from the reference counts by the test.
  group_c0.npz      the reference per-group call for one customer / one terminal (frame
                    layout contract: row order, index = TRANSACTION_ID, column order).
  forest_*.npz      sklearn DecisionTree(depth 2) / RandomForest(5, depth 8) / RF(3 trees,
                    unlimited depth) trained like model_training.ipynb (scaleData, then fit)
                    on tiny features: node arrays + scaler + test X (with NaN rows, the
                    Spark LEFT JOIN NULL case) + expected tree_.apply leaf ids and
                    predict_proba[:, 1].
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden")

FEATURES = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT",
            "CUSTOMER_ID_NB_TX_1DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_1DAY_WINDOW",
            "CUSTOMER_ID_NB_TX_7DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_7DAY_WINDOW",
            "CUSTOMER_ID_NB_TX_30DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_30DAY_WINDOW",
            "TERMINAL_ID_NB_TX_1DAY_WINDOW", "TERMINAL_ID_RISK_1DAY_WINDOW",
            "TERMINAL_ID_NB_TX_7DAY_WINDOW", "TERMINAL_ID_RISK_7DAY_WINDOW",
            "TERMINAL_ID_NB_TX_30DAY_WINDOW", "TERMINAL_ID_RISK_30DAY_WINDOW"]


def _ns(series):
    return series.values.astype("datetime64[ns]").astype(np.int64)


def save_table(path, df):
    out = dict(
        TRANSACTION_ID=df.TRANSACTION_ID.values.astype(np.int64),
        TX_DATETIME=_ns(df.TX_DATETIME),
        CUSTOMER_ID=df.CUSTOMER_ID.values.astype(np.int64),
        TERMINAL_ID=df.TERMINAL_ID.values.astype(np.int64),
        TX_AMOUNT=df.TX_AMOUNT.values.astype(np.float64),
        TX_FRAUD=df.TX_FRAUD.values.astype(np.int64),
    )
    for c in FEATURES[1:]:
        out[c] = df[c].values.astype(np.float64)
    np.savez_compressed(path, **out)


def main():
    warnings.filterwarnings("ignore")
    sys.path.insert(0, HERE)
    import pandas as pd
    import sklearn.ensemble
    import sklearn.tree
    import refexec

    os.makedirs(GOLDEN, exist_ok=True)
    ns = refexec.load_namespace()
    tables = {}
    for name, (nc, nt, nd, r) in {"a": (120, 300, 60, 8), "b": (25, 10, 75, 60)}.items():
        c, t, df = ns["generate_dataset"](n_customers=nc, n_terminals=nt, nb_days=nd,
                                          start_date="2024-06-01", r=r)
        df = ns["add_frauds"](c, t, df)
        df = df.replace([-1], 0)  # read_from_files normalisation (shared_functions.py:88)
        for col in ("CUSTOMER_ID", "TERMINAL_ID", "TX_TIME_SECONDS", "TX_TIME_DAYS"):
            df[col] = df[col].astype(np.int64)
        raw = df.copy()
        feat = refexec.reference_featurize(ns, df)
        save_table(os.path.join(GOLDEN, f"tiny_{name}.npz"), feat)
        tables[name] = (raw, feat)
        print(name, feat.shape, int(feat.TX_FRAUD.sum()))

    # tie-heavy table: timestamps floored to the hour (many equal (customer, time) pairs)
    raw = tables["b"][0].copy()
    raw["TX_DATETIME"] = raw["TX_DATETIME"].dt.floor("h")
    raw = raw.sort_values("TX_DATETIME", kind="stable").reset_index(drop=True)
    raw["TRANSACTION_ID"] = np.arange(len(raw))
    feat = refexec.reference_featurize(ns, raw)
    save_table(os.path.join(GOLDEN, "ties.npz"), feat)
    print("ties", feat.shape)

    # per-group call contract (one customer, one terminal), columns in reference order
    raw, feat = tables["a"]
    g = raw[raw.CUSTOMER_ID == raw.CUSTOMER_ID.iloc[0]].copy()
    g["TX_DURING_WEEKEND"] = g.TX_DATETIME.apply(ns["is_weekend"])
    g["TX_DURING_NIGHT"] = g.TX_DATETIME.apply(ns["is_night"])
    oc = ns["get_customer_spending_behaviour_features"](g, windows_size_in_days=[1, 7, 30])
    tt = feat[feat.TERMINAL_ID == feat.TERMINAL_ID.iloc[0]].copy()
    ot = ns["get_count_risk_rolling_window"](tt.drop(columns=[c for c in tt.columns if c.startswith("TERMINAL_ID_")]),
                                             delay_period=7, windows_size_in_days=[1, 7, 30], feature="TERMINAL_ID")
    np.savez_compressed(
        os.path.join(GOLDEN, "group_c0.npz"),
        cust_columns=np.array(list(oc.columns)), cust_index=oc.index.values.astype(np.int64),
        cust_values=oc[[c for c in oc.columns if c.startswith("CUSTOMER_ID_")]].values,
        cust_in_tid=g.TRANSACTION_ID.values.astype(np.int64),
        term_columns=np.array(list(ot.columns)), term_index=ot.index.values.astype(np.int64),
        term_values=ot[[c for c in ot.columns if c.startswith("TERMINAL_ID_")]].values,
        term_in_tid=tt.TRANSACTION_ID.values.astype(np.int64),
    )

    # forests, trained as model_training.ipynb does (scaleData then fit on the train days)
    feat = tables["a"][1]
    days = (feat.TX_DATETIME - feat.TX_DATETIME.min()).dt.days.values
    train, test = feat[days < 40].copy(), feat[days >= 40].copy()
    train, test, scaler = ns["scaleData"](train, test, FEATURES)
    Xtest_raw = tables["a"][1][days >= 40][FEATURES].values.astype(np.float64)
    rng = np.random.RandomState(0)
    Xnan = Xtest_raw[:64].copy()
    Xnan[rng.rand(*Xnan.shape) < 0.2] = np.nan  # Spark LEFT JOIN misses -> NULL -> NaN
    Xall = np.vstack([Xtest_raw, Xnan])
    Zall = scaler.transform(pd.DataFrame(Xall, columns=FEATURES))
    models = {
        "dt2": sklearn.tree.DecisionTreeClassifier(max_depth=2, random_state=0),
        "rf5d8": sklearn.ensemble.RandomForestClassifier(n_estimators=5, max_depth=8, random_state=0, n_jobs=1),
        "rf3": sklearn.ensemble.RandomForestClassifier(n_estimators=3, random_state=0, n_jobs=1),
    }
    for name, m in models.items():
        m.fit(train[FEATURES], train["TX_FRAUD"])
        ests = getattr(m, "estimators_", [m])
        off = np.cumsum([0] + [e.tree_.node_count for e in ests])
        cat = lambda f: np.concatenate([f(e.tree_) for e in ests])
        Zdf = pd.DataFrame(Zall, columns=FEATURES)
        leaves = np.stack([e.tree_.apply(Zdf.values.astype(np.float32)) for e in ests], axis=1)
        np.savez_compressed(
            os.path.join(GOLDEN, f"forest_{name}.npz"),
            node_offsets=off.astype(np.int64),
            left=cat(lambda t: t.children_left).astype(np.int64),
            right=cat(lambda t: t.children_right).astype(np.int64),
            feature=cat(lambda t: t.feature).astype(np.int64),
            threshold=cat(lambda t: t.threshold).astype(np.float64),
            missing_left=cat(lambda t: np.asarray(t.missing_go_to_left)).astype(np.uint8),
            value1=cat(lambda t: t.value[:, 0, 1]).astype(np.float64),
            mean=scaler.mean_, scale=scaler.scale_, X=Xall,
            leaves=leaves.astype(np.int32), proba=m.predict_proba(Zdf)[:, 1],
        )
        print(name, off[-1], "nodes")


if __name__ == "__main__":
    main()
