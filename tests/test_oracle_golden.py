"""The CPU oracle against the reference's golden vectors (no GPU).

Pins the oracle before it is trusted as the checker of the HIP path:
  * tiny_a / tiny_b: every derived column, bit-exact, vs the reference's notebook
    functions run on the reference generator's data (oracle/gen_golden.py);
  * ties: (CUSTOMER_ID, TX_DATETIME) ties -- pandas' per-group quicksort order is
    recovered from the reference counts, then exact;
  * notebook_kat: values printed in the committed notebook outputs
    (feature_transformation.ipynb cells 19/22/29/32/36/43/51/54) to the printed decimals;
  * forest_*: sklearn apply() leaf ids and predict_proba[:, 1], bit-exact.
"""
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

ALL_COLS = ["TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + oracle.CUSTOMER_COLS + oracle.TERMINAL_COLS


@pytest.mark.parametrize("name", ["tiny_a.npz", "tiny_b.npz"])
def test_oracle_matches_reference_tables(golden, name):
    z = golden(name)
    order = np.argsort(z["TRANSACTION_ID"], kind="stable")
    f = oracle.featurize_arrays(z["TX_DATETIME"][order], z["CUSTOMER_ID"][order], z["TERMINAL_ID"][order],
                                z["TX_AMOUNT"][order], z["TX_FRAUD"][order])
    for c in ALL_COLS:
        np.testing.assert_array_equal(f[c].astype(np.float64), z[c][order], err_msg=c)


def _tie_aware_customer_order(z):
    """Rows grouped by customer, time order, tied rows in the reference's processing order
    (NB_TX is strictly increasing along the processing order inside a tie group)."""
    return np.lexsort((z["CUSTOMER_ID_NB_TX_1DAY_WINDOW"], z["TX_DATETIME"], z["CUSTOMER_ID"]))


def test_oracle_ties(golden):
    z = golden("ties.npz")
    key = z["CUSTOMER_ID"] * (1 << 40) + z["TX_DATETIME"] // 10**9
    _, counts = np.unique(key, return_counts=True)
    assert (counts > 1).sum() > 20, "fixture must contain tie groups"
    order = _tie_aware_customer_order(z)
    sk = z["CUSTOMER_ID"][order]
    seg = np.r_[np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]]), len(sk)]
    nb, avg = oracle.customer_windows(z["TX_DATETIME"][order], z["TX_AMOUNT"][order], seg)
    for k, w in enumerate((1, 7, 30)):
        np.testing.assert_array_equal(nb[k], z[f"CUSTOMER_ID_NB_TX_{w}DAY_WINDOW"][order])
        np.testing.assert_array_equal(avg[k], z[f"CUSTOMER_ID_AVG_AMOUNT_{w}DAY_WINDOW"][order])
    # terminal features do not depend on tie order
    f = oracle.featurize_arrays(z["TX_DATETIME"], z["CUSTOMER_ID"], z["TERMINAL_ID"], z["TX_AMOUNT"],
                                z["TX_FRAUD"])
    for c in oracle.TERMINAL_COLS:
        np.testing.assert_array_equal(f[c], z[c], err_msg=c)


def test_oracle_notebook_known_answers():
    from kat_check import check_notebook_kat

    check_notebook_kat(lambda ts, c, t, a, fr, tids: oracle.featurize_arrays(ts, c, t, a, fr))


@pytest.mark.parametrize("name", ["forest_dt2.npz", "forest_rf5d8.npz", "forest_rf3.npz"])
def test_oracle_forest_matches_sklearn(golden, name):
    z = golden(name)
    arrays = {k: z[k] for k in ("left", "right", "feature", "threshold", "missing_left", "value1", "node_offsets")}
    proba, leaves = oracle.forest_predict(z["X"], arrays, z["mean"], z["scale"], want_leaves=True)
    np.testing.assert_array_equal(leaves, z["leaves"])
    np.testing.assert_array_equal(proba, z["proba"])
    assert np.isnan(z["X"]).any()


def test_spark_flag_semantics():
    # 2024-06-01 is a Saturday; Spark dayofweek: Sunday=1 .. Saturday=7
    base = np.datetime64("2024-06-01T00:00:00", "ns").astype(np.int64)
    day = 86_400 * 10**9
    ts = np.array([base + k * day + 21 * 3600 * 10**9 for k in range(7)])  # Sat..Fri at 21:00
    np.testing.assert_array_equal(oracle.weekend_flag(ts), [1, 1, 0, 0, 0, 0, 0])
    np.testing.assert_array_equal(oracle.spark_weekend_flag(ts), [1, 0, 0, 0, 0, 1, 1])  # Sat, Thu, Fri
    np.testing.assert_array_equal(oracle.spark_night_flag(ts), [1] * 7)
    np.testing.assert_array_equal(oracle.night_flag(ts), [0] * 7)
