"""Host-side helpers of bench.py (no GPU): the forest's walk-step count used by the LDS
roofline."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_walk_steps_per_row_sums_tree_depths():
    b = _bench()
    # tree 0: root -> (leaf, node -> (leaf, leaf)): depth 2; tree 1: a single leaf: depth 0;
    # tree 2: root -> (leaf, leaf): depth 1   (pre-order, -1 = leaf, per-tree local ids)
    left = np.array([1, -1, 3, -1, -1, -1, 1, -1, -1])
    right = np.array([2, -1, 4, -1, -1, -1, 2, -1, -1])
    off = np.array([0, 5, 6, 9])
    assert b.walk_steps_per_row({"left": left, "right": right, "node_offsets": off}) == 3


def test_walk_steps_of_the_bench_model():
    b = _bench()
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    a = {k: z[k] for k in ("left", "right", "node_offsets")}
    assert b.walk_steps_per_row(a) == 2000  # 100 trees, every one reaches depth 20
    assert b.LDS_PEAK_STEPS == 256 * 2.4e9 / 4 * 64


def test_sklearn_forest_rebuilt_from_arrays_matches_saved_output():
    """The CPU baseline times scikit-learn itself on the bench model, rebuilt from its node
    arrays (no pickle): the rebuilt forest must give sklearn's saved predict_proba bit for bit."""
    import sklearn.preprocessing

    b = _bench()
    arrays, mean, scale, cx, cp = b.load_model(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    rf = b.sklearn_forest(arrays)
    sc = sklearn.preprocessing.StandardScaler()
    sc.mean_, sc.scale_, sc.var_, sc.n_features_in_, sc.n_samples_seen_ = mean, scale, scale * scale, 15, 1
    rf.set_params(n_jobs=1)
    np.testing.assert_array_equal(rf.predict_proba(sc.transform(cx[:512]))[:, 1], cp[:512])


def test_host_info_fields():
    info = _bench().host_info()
    assert info["nproc"] >= 1 and info["affinity_cpus"] >= 1 and info["joblib_cpus"] >= 1
