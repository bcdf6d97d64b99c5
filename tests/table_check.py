"""Host-side reading of the featurized table that the scoring path's assembly pass writes
(run_fused(rows_out=ops.FeatureTable(...)), feature_transformation.ipynb:2890-2905's 14 derived
columns by scoring slot).  Test helper: the product never reads its own table back."""
import numpy as np


def table_as_X(rows, n_slots: int, amount) -> np.ndarray:
    """FeatureTable (slot order) -> the [n, 15] float64 input_features matrix in input row order
    (column 0 = TX_AMOUNT from the caller's input, which the table does not repeat).  Asserts the
    table's own invariants first: every input row in exactly one slot, padding slots row -1 with
    zero features."""
    n = len(amount)
    col = {k: v.cpu().numpy() for k, v in rows.columns(n_slots).items()}
    real = col["row"] >= 0
    assert int(real.sum()) == n, (int(real.sum()), n)
    assert not col["cust_nb"][:, ~real].any() and not col["term_nb"][:, ~real].any()
    assert not col["cust_avg"][:, ~real].any() and not col["term_risk"][:, ~real].any()
    assert not col["weekend"][~real].any() and not col["night"][~real].any()
    r = col["row"][real]
    X = np.zeros((n, 15), np.float64)
    seen = np.zeros(n, np.int64)
    np.add.at(seen, r, 1)
    assert (seen == 1).all(), "a row is missing from the table or written twice"
    X[:, 0] = amount
    X[r, 1] = col["weekend"][real]
    X[r, 2] = col["night"][real]
    for w in range(3):
        X[r, 3 + 2 * w] = col["cust_nb"][w][real]
        X[r, 4 + 2 * w] = col["cust_avg"][w][real]
        X[r, 9 + 2 * w] = col["term_nb"][w][real]
        X[r, 10 + 2 * w] = col["term_risk"][w][real]
    return X


def assert_same_features(got: np.ndarray, want: np.ndarray, what: str = ""):
    """Columns 1..14 bit for bit (float columns compared as their IEEE bit patterns)."""
    assert got.shape == want.shape, (got.shape, want.shape)
    for j in range(1, 15):
        np.testing.assert_array_equal(np.ascontiguousarray(got[:, j]).view(np.int64),
                                      np.ascontiguousarray(want[:, j]).view(np.int64),
                                      err_msg=f"{what} column {j}")
