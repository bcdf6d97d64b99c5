"""The bench / large-test input generator (fdx/synth.py) keeps the handbook generator's
terminal choice: uniform among the terminals strictly within radius r of the customer
(data_generator.ipynb:420-437, :821)."""
import numpy as np

from fdx import synth


def test_terminal_sampler_is_uniform_within_radius():
    trng = np.random.default_rng(3)
    tx, ty = trng.uniform(0, 100, 5000), trng.uniform(0, 100, 5000)
    s = synth._TerminalSampler(tx, ty, 5.0)
    rng = np.random.default_rng(4)
    for px, py in ((50.0, 50.0), (1.0, 2.0), (99.5, 40.0), (30.0, 97.0)):
        inside = np.flatnonzero(np.sqrt((tx - px) ** 2 + (ty - py) ** 2) < 5.0)
        m = 100_000
        P, Q = np.full(m, px), np.full(m, py)
        lo, hi = s.ranges(P[:1], Q[:1])
        got = s.sample(rng, P, Q, np.repeat(lo, m, 0), np.repeat(hi, m, 0))
        assert np.isin(got, inside).all()
        cnt = np.bincount(got, minlength=len(tx))[inside]
        exp = m / len(inside)
        assert (cnt > 0).all()
        assert np.abs(cnt - exp).max() < 6 * np.sqrt(exp)
    assert s.has_terminal(np.array([50.0]), np.array([50.0]))[0]


def test_generate_shape_and_order():
    d = synth.generate(n_customers=300, n_terminals=600, nb_days=20, seed=1)
    assert (np.diff(d["ts"]) >= 0).all()
    assert d["customer"].max() < 300 and d["terminal"].max() < 600
    assert set(np.unique(d["fraud"])) <= {0, 1}


def test_numpy_generator_matches_reference_statistics_config1():
    """fdx.synth at BASELINE config 1 (5k customers / 10k terminals / 183 days) against the
    reference generator's own output: 1,754,155 tx, 14,681 frauds (973 / 9,076 / 4,632 by
    scenario), amount and time-of-day moments, per-customer volume quantiles."""
    import synth_stats
    from fdx import synth

    for seed in (0, 1):
        d = synth.generate(5000, 10000, 183, seed=seed)
        secs = (d["ts"] - synth.START_NS) // synth.NS
        synth_stats.assert_close(synth_stats.stats(d["day"], secs, d["customer"], d["terminal"], d["amount"],
                                                   d["fraud"], d["scenario"]))
