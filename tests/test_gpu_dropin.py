"""The pandas / sklearn drop-ins (fdx.*) against the reference's contracts and outputs."""
import numpy as np
import pandas as pd
import pytest

import fdx
import oracle

pytestmark = pytest.mark.gpu

CUST = ["CUSTOMER_ID_NB_TX_1DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_1DAY_WINDOW", "CUSTOMER_ID_NB_TX_7DAY_WINDOW",
        "CUSTOMER_ID_AVG_AMOUNT_7DAY_WINDOW", "CUSTOMER_ID_NB_TX_30DAY_WINDOW",
        "CUSTOMER_ID_AVG_AMOUNT_30DAY_WINDOW"]
TERM = [c.replace("CUSTOMER_ID_AVG_AMOUNT", "TERMINAL_ID_RISK").replace("CUSTOMER_ID", "TERMINAL_ID") for c in CUST]


def _frame(z, tids=None):
    df = pd.DataFrame({
        "TRANSACTION_ID": z["TRANSACTION_ID"],
        "TX_DATETIME": pd.to_datetime(z["TX_DATETIME"], unit="ns"),
        "CUSTOMER_ID": z["CUSTOMER_ID"], "TERMINAL_ID": z["TERMINAL_ID"],
        "TX_AMOUNT": z["TX_AMOUNT"], "TX_FRAUD": z["TX_FRAUD"],
    }).sort_values("TRANSACTION_ID").reset_index(drop=True)
    if tids is not None:
        df = df[df.TRANSACTION_ID.isin(tids)]
    return df


def test_customer_group_call_contract(golden):
    z, g = golden("tiny_a.npz"), golden("group_c0.npz")
    df = _frame(z, g["cust_in_tid"])
    out = fdx.get_customer_spending_behaviour_features(df, windows_size_in_days=[1, 7, 30])
    assert list(out.columns) == list(df.columns) + CUST
    assert out.index.name == "TRANSACTION_ID"
    np.testing.assert_array_equal(out.index.values, g["cust_index"])
    np.testing.assert_array_equal(out[CUST].values, g["cust_values"])
    assert all(out[c].dtype == np.float64 for c in CUST)


def test_terminal_group_call_contract(golden):
    z, g = golden("tiny_a.npz"), golden("group_c0.npz")
    df = _frame(z, g["term_in_tid"])
    out = fdx.get_count_risk_rolling_window(df, delay_period=7, windows_size_in_days=[1, 7, 30],
                                            feature="TERMINAL_ID")
    assert list(out.columns) == list(df.columns) + TERM
    np.testing.assert_array_equal(out.index.values, g["term_index"])
    np.testing.assert_array_equal(out[TERM].values, g["term_values"])


@pytest.mark.parametrize("shuffle", [False, True])
def test_whole_frame_equals_groupby_apply(golden, shuffle):
    """One call on the whole frame == the notebook's groupby.apply + sort (values by tid)."""
    z = golden("tiny_b.npz")
    df = _frame(z)
    if shuffle:
        df = df.sample(frac=1.0, random_state=0)
    out = fdx.get_customer_spending_behaviour_features(df)
    out = out.sort_values("TX_DATETIME", kind="stable").reset_index(drop=True)
    out = fdx.get_count_risk_rolling_window(out, delay_period=7, windows_size_in_days=[1, 7, 30])
    out = out.set_index("TRANSACTION_ID").sort_index()
    order = np.argsort(z["TRANSACTION_ID"])
    for c in CUST + TERM:
        np.testing.assert_array_equal(out[c].values, z[c][order], err_msg=c)
    # groups come out in key order, time order inside
    grp = fdx.get_customer_spending_behaviour_features(df)
    assert (np.diff(grp.CUSTOMER_ID.values) >= 0).all()


def test_flags_dropin(golden):
    z = golden("tiny_a.npz")
    s = pd.Series(pd.to_datetime(z["TX_DATETIME"], unit="ns"))
    np.testing.assert_array_equal(fdx.is_weekend(s).values, z["TX_DURING_WEEKEND"])
    np.testing.assert_array_equal(fdx.is_night(s).values, z["TX_DURING_NIGHT"])
    assert fdx.is_weekend(pd.Timestamp("2024-06-01 10:00")) == 1
    assert fdx.is_night(pd.Timestamp("2024-06-03 06:59:59")) == 1
    assert fdx.is_night(pd.Timestamp("2024-06-03 07:00:00")) == 0
    assert fdx.is_weekend(pd.Timestamp("2024-06-06 10:00"), mode=fdx.FDX_FLAGS_SPARK) == 1  # Thursday


def test_fit_model_and_get_predictions_matches_sklearn(golden):
    import sklearn.ensemble
    import sklearn.tree

    z = golden("tiny_a.npz")
    df = pd.DataFrame({c: z[c] for c in fdx.INPUT_FEATURES[1:]})
    df.insert(0, "TX_AMOUNT", z["TX_AMOUNT"])
    df["TX_FRAUD"] = z["TX_FRAUD"]
    train, test = df.iloc[: len(df) * 2 // 3].copy(), df.iloc[len(df) * 2 // 3:].copy()
    for clf_gpu, clf_cpu in (
        (sklearn.tree.DecisionTreeClassifier(max_depth=2, random_state=0),
         sklearn.tree.DecisionTreeClassifier(max_depth=2, random_state=0)),
        (sklearn.ensemble.RandomForestClassifier(n_estimators=10, max_depth=12, random_state=0, n_jobs=1),
         sklearn.ensemble.RandomForestClassifier(n_estimators=10, max_depth=12, random_state=0, n_jobs=1))):
        res = fdx.fit_model_and_get_predictions(clf_gpu, train.copy(), test.copy(), fdx.INPUT_FEATURES)
        assert set(res) == {"classifier", "predictions_test", "predictions_train", "training_execution_time",
                            "prediction_execution_time"}
        tr, te = train.copy(), test.copy()
        import sklearn.preprocessing
        sc = sklearn.preprocessing.StandardScaler().fit(tr[fdx.INPUT_FEATURES])
        tr[fdx.INPUT_FEATURES] = sc.transform(tr[fdx.INPUT_FEATURES])
        te[fdx.INPUT_FEATURES] = sc.transform(te[fdx.INPUT_FEATURES])
        clf_cpu.fit(tr[fdx.INPUT_FEATURES], tr["TX_FRAUD"])
        np.testing.assert_array_equal(res["predictions_test"], clf_cpu.predict_proba(te[fdx.INPUT_FEATURES])[:, 1])
        np.testing.assert_array_equal(res["predictions_train"], clf_cpu.predict_proba(tr[fdx.INPUT_FEATURES])[:, 1])
        g = fdx.GpuForest(res["classifier"])
        np.testing.assert_array_equal(g.apply(te[fdx.INPUT_FEATURES]),
                                      np.asarray(res["classifier"].apply(te[fdx.INPUT_FEATURES])).reshape(len(te), -1))


def test_spark_udf_body(golden):
    """fraud_detection.py:183-195 with Spark-shaped inputs: int32 counts, Decimal amounts,
    NULL (NaN) features from LEFT JOIN misses."""
    import decimal

    import sklearn.ensemble
    import sklearn.preprocessing

    z = golden("tiny_a.npz")
    X = np.column_stack([z["TX_AMOUNT"]] + [z[c] for c in fdx.INPUT_FEATURES[1:]])
    sc = sklearn.preprocessing.StandardScaler().fit(X)
    rf = sklearn.ensemble.RandomForestClassifier(n_estimators=8, max_depth=10, random_state=0, n_jobs=1)
    rf.fit(sc.transform(X), z["TX_FRAUD"])
    udf = fdx.make_scale_and_predict_udf(rf, sc)
    n = 3000
    cols = [pd.Series([decimal.Decimal(f"{a:.2f}") for a in z["TX_AMOUNT"][:n]])]
    for j, c in enumerate(fdx.INPUT_FEATURES[1:]):
        v = z[c][:n].copy()
        if "NB_TX" in c or "DURING" in c:
            s = pd.Series(v.astype(np.int32))
        else:
            s = pd.Series(v)
        if j % 4 == 0:
            s = s.astype(np.float64)
            s.iloc[::37] = np.nan
        cols.append(s)
    got = udf(*cols)
    feats = pd.concat(cols, axis=1)
    feats.columns = fdx.INPUT_FEATURES
    feats["TX_AMOUNT"] = feats["TX_AMOUNT"].astype(np.float64)
    exp = rf.predict_proba(sc.transform(feats))[:, 1]
    assert isinstance(got, pd.Series) and got.dtype == np.float64
    np.testing.assert_array_equal(got.values, exp)
    _ = oracle


def test_model_zoo_non_tree_classifier_uses_own_predict_proba(golden):
    """model_training.ipynb:2209-2223 loops over LR, DT, RF, XGB: the drop-in must not break
    on LogisticRegression (its own predict_proba on the GPU-scaled frame)."""
    import sklearn.linear_model
    import sklearn.preprocessing

    z = golden("tiny_a.npz")
    df = pd.DataFrame({c: z[c] for c in fdx.INPUT_FEATURES[1:]})
    df.insert(0, "TX_AMOUNT", z["TX_AMOUNT"])
    df["TX_FRAUD"] = z["TX_FRAUD"]
    train, test = df.iloc[: len(df) * 2 // 3].copy(), df.iloc[len(df) * 2 // 3:].copy()
    res = fdx.fit_model_and_get_predictions(sklearn.linear_model.LogisticRegression(max_iter=200), train.copy(),
                                            test.copy(), fdx.INPUT_FEATURES)
    tr, te = train.copy(), test.copy()
    sc = sklearn.preprocessing.StandardScaler().fit(tr[fdx.INPUT_FEATURES])
    tr[fdx.INPUT_FEATURES] = sc.transform(tr[fdx.INPUT_FEATURES])
    te[fdx.INPUT_FEATURES] = sc.transform(te[fdx.INPUT_FEATURES])
    lr = sklearn.linear_model.LogisticRegression(max_iter=200).fit(tr[fdx.INPUT_FEATURES], tr["TX_FRAUD"])
    np.testing.assert_array_equal(res["predictions_test"], lr.predict_proba(te[fdx.INPUT_FEATURES])[:, 1])
    # the UDF body with a non-tree model: GPU scaling, then the model's own predict_proba
    udf = fdx.make_scale_and_predict_udf(lr, sc)
    cols = [pd.Series(test[c].values) for c in fdx.INPUT_FEATURES]
    np.testing.assert_array_equal(udf(*cols).values, lr.predict_proba(sc.transform(test[fdx.INPUT_FEATURES]))[:, 1])


def test_predict_proba_both_columns_bit_exact(golden):
    """GpuForest.predict_proba: column 0 is sklearn's tree-order sum of value[:, 0, 0], not 1 - p."""
    import sklearn.ensemble

    z = golden("tiny_a.npz")
    X = np.column_stack([z["TX_AMOUNT"]] + [z[c] for c in fdx.INPUT_FEATURES[1:]])
    rf = sklearn.ensemble.RandomForestClassifier(n_estimators=7, max_depth=9, random_state=0, n_jobs=1)
    rf.fit(X[:6000], z["TX_FRAUD"][:6000])
    got = fdx.GpuForest(rf).predict_proba(X[6000:])
    np.testing.assert_array_equal(got, rf.predict_proba(X[6000:].astype(np.float32)))


def test_sparse_and_negative_ids_group_like_pandas(golden):
    """Ids that are not dense (huge, negative, gappy) take the sort-based dense re-id on the GPU
    (fdx_dense_ids_i64): the features must equal those of the same frame with dense ids."""
    z = golden("tiny_b.npz")
    df = _frame(z)
    rng = np.random.default_rng(11)
    for col in ("CUSTOMER_ID", "TERMINAL_ID"):
        ids = np.unique(df[col].values)
        sparse = np.sort(rng.choice(np.arange(-(1 << 40), 1 << 40, 7919, dtype=np.int64), len(ids), replace=False))
        remap = dict(zip(ids, sparse))
        ds = df.copy()
        ds[col] = ds[col].map(remap).astype(np.int64)
        if col == "CUSTOMER_ID":
            a = fdx.get_customer_spending_behaviour_features(df)[CUST].sort_index()
            b = fdx.get_customer_spending_behaviour_features(ds)[CUST].sort_index()
        else:
            a = fdx.get_count_risk_rolling_window(df)[TERM].sort_index()
            b = fdx.get_count_risk_rolling_window(ds)[TERM].sort_index()
        np.testing.assert_array_equal(a.values, b.values)


def test_dense_ids_i64_kernel(dev):
    import torch

    from fdx import ops

    rng = np.random.default_rng(5)
    for n in (1, 7, 100_003):
        k = rng.integers(-(1 << 62), 1 << 62, n // 3 + 1)[rng.integers(0, n // 3 + 1, n)]
        ids, nu = ops.dense_ids_i64(torch.from_numpy(k).to(dev))
        u, inv = np.unique(k, return_inverse=True)
        np.testing.assert_array_equal(ids.cpu().numpy(), inv.astype(np.int32))
        assert int(nu.item()) == len(u)
    ids, nu = ops.dense_ids_i64(torch.empty(0, dtype=torch.int64, device=dev))
    assert ids.numel() == 0 and int(nu.item()) == 0
