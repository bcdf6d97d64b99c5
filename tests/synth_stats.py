"""Config-1 statistics of a generated table against the reference generator's
(tests/golden/config1_stats.json, written by oracle/gen_synth_stats.py from the reference's
own generate_dataset + add_frauds).  The generators reproduce the distributions, not the
reference's RNG stream, so each statistic is compared within a tolerance of about 4-5 standard
deviations of its seed-to-seed spread (measured over 6 seeds of fdx.synth at config 1:
n_tx sd 0.55 %, n_fraud sd 2.2 %, scenario 1/2/3 sd 5 % / 2.3 % / 2 %, amount mean sd 1.1 %,
amount sd sd 0.4 %, customer-count quantiles sd <= 3 %, second-of-day mean sd 0.04 %).
Scenario 3 draws a Bernoulli(1/3) per compromised row where the reference samples exactly a
third per compromised customer-day batch -- same expectation."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TOL = {"n_tx": 0.03, "n_fraud": 0.10, "tx_per_customer_day": 0.03, "amount_mean": 0.05, "amount_std": 0.03,
       "genuine_amount_mean": 0.05, "second_of_day_mean": 0.003, "second_of_day_std": 0.01, "night_share": 0.03}
TOL_Q = [0.35, 0.10, 0.06, 0.05, 0.03]
TOL_SCEN = {"1": 0.25, "2": 0.12, "3": 0.12}


def reference():
    with open(os.path.join(HERE, "golden", "config1_stats.json")) as f:
        return json.load(f)


def stats(day, secs, cust, term, amount, fraud, scenario, n_customers=5000, nb_days=183):
    import sys

    sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
    from gen_synth_stats import stats_of

    return stats_of(np.asarray(day, np.int64), np.asarray(secs, np.int64), np.asarray(cust, np.int64),
                    np.asarray(term, np.int64), np.asarray(amount, np.float64), np.asarray(fraud, np.int64),
                    None if scenario is None else np.asarray(scenario, np.int64), n_customers, nb_days)


def assert_close(got, ref=None):
    ref = ref or reference()
    bad = []
    for k, tol in TOL.items():
        if abs(got[k] / ref[k] - 1) > tol:
            bad.append(f"{k}: {got[k]:.6g} vs reference {ref[k]:.6g} (tol {tol:.0%})")
    for i, tol in enumerate(TOL_Q):
        if abs(got["per_customer_tx_q"][i] / ref["per_customer_tx_q"][i] - 1) > tol:
            bad.append(f"per-customer tx quantile {i}: {got['per_customer_tx_q'][i]} vs {ref['per_customer_tx_q'][i]}")
    for s, tol in TOL_SCEN.items():
        g, r = got["scenario_counts"][s], ref["scenario_counts"][s]
        if abs(g / r - 1) > tol:
            bad.append(f"scenario {s}: {g} vs {r} (tol {tol:.0%})")
    if got["terminals_used"] != ref["terminals_used"]:
        bad.append(f"terminals used {got['terminals_used']} vs {ref['terminals_used']}")
    assert not bad, "; ".join(bad)
