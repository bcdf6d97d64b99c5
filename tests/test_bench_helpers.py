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


def test_plan_workload_configs1_at_one_gpu():
    b = _bench()
    w = b.plan_workload(1, 0)
    assert w["name"] == "configs1" and w["scaling"] == "weak"
    assert (w["customer_base"], w["n_customers_local"], w["n_terminals_total"], w["days"]) == (0, 50_000, 100_000, 183)


def test_plan_workload_configs3_strong_scaling_over_8_ranks():
    """bench.py --gpus 8 runs BASELINE.json configs[3]: 1M customers / 2M terminals / 365 days in
    total, contiguous customer ranges, the terminal id space independent of N."""
    b = _bench()
    for world in (2, 4, 8):
        plans = [b.plan_workload(world, r) for r in range(world)]
        assert all(p["name"] == "configs3" and p["scaling"] == "strong" for p in plans)
        assert all(p["n_terminals_total"] == 2_000_000 and p["days"] == 365 for p in plans)
        assert plans[0]["customer_base"] == 0
        for a, c in zip(plans, plans[1:]):
            assert a["customer_base"] + a["n_customers_local"] == c["customer_base"]
        assert sum(p["n_customers_local"] for p in plans) == 1_000_000
    p8 = [b.plan_workload(8, r) for r in range(8)]
    assert [(p["customer_base"], p["n_customers_local"]) for p in p8] == [(r * 125_000, 125_000) for r in range(8)]


def test_stage_table_medians_and_rejects_inflated_isolated_times():
    """An isolated stage time more than 2x its in-step time (BENCH_r03: one cold step of 15-21 ms
    folded into a mean of 3) is rejected: the roofline uses the in-step median instead."""
    b = _bench()
    stages = [("rekey_customer", "K2", []), ("customer_walk", "K1-cust", []), ("forest_traverse", "K3", [])]
    in_step = {"rekey_customer": [0.9, 0.95, 1.0], "customer_walk": [1.0, 1.0, 1.1], "forest_traverse": [7.2, 7.1, 7.3]}
    iso = {"rekey_customer": [0.58, 15.9, 0.59], "customer_walk": [21.0, 22.0, 0.75], "forest_traverse": [7.0, 7.1, 7.2]}
    rows = {r["stage"]: r for r in b.stage_table(in_step, iso, stages)}
    assert rows["rekey_customer"]["ms"] == 0.59 and rows["rekey_customer"]["ms_isolated"] == 0.59  # median
    assert "ms_isolated" not in rows["customer_walk"]
    assert rows["customer_walk"]["ms_isolated_rejected"] == 21.0
    assert rows["customer_walk"]["ms"] == rows["customer_walk"]["ms_in_step"] == 1.0
    assert rows["forest_traverse"]["ms"] == 7.1
    assert b.stage_table(in_step, None, stages)[0]["ms"] == 0.95


def test_bench_stream_splits_configs4_state_over_ranks():
    """bench_stream.py --gpus N: the 1M / 2M-key state of configs[4] split over the ranks --
    contiguous customer ranges covering every id once, every rank with all terminal ids."""
    import bench_stream

    a = bench_stream.parse([])
    assert (a.customers, a.terminals, a.batch) == (1_000_000, 2_000_000, 65536)
    for world in (1, 2, 4, 8):
        shards = [bench_stream.rank_shard(a, world, r) for r in range(world)]
        covered = np.concatenate([np.arange(base, base + n_c) for n_c, base, _ in shards])
        np.testing.assert_array_equal(covered, np.arange(1_000_000))
        assert all(t == 2_000_000 for _, _, t in shards)
