"""Reference statistics of the handbook generator at config 1 (TEST INFRASTRUCTURE ONLY).

Runs the reference's own generator (data_generator.ipynb generate_dataset :1339-1371 +
add_frauds :1732-1782, exec'd from the notebook by oracle/refexec.py, build container only)
for BASELINE.json configs[0] -- 5,000 customers / 10,000 terminals, seeds as the notebook --
keeps the first 183 days (identical to a 183-day run: the RNG is seeded per customer and
consumed day by day) and writes summary statistics to
tests/golden/config1_stats.json.  fdx.synth (numpy) and the HIP generator
(csrc/fdx_synth.hip) are checked against them within sampling error
(tests/test_synth.py, tests/test_gpu_synth.py): they reproduce the distributions, not the
reference's Python RNG stream.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def stats_of(day, secs, cust, term, amount, fraud, scenario, n_customers, nb_days):
    """The statistics compared (scenario may be None: only the totals then)."""
    per_c = np.bincount(cust, minlength=n_customers)
    sod = secs - day * 86400
    out = {
        "n_tx": int(len(day)),
        "n_fraud": int(fraud.sum()),
        "tx_per_customer_day": float(len(day) / (n_customers * nb_days)),
        "per_customer_tx_q": [float(q) for q in np.quantile(per_c, [0.05, 0.25, 0.5, 0.75, 0.95])],
        "amount_mean": float(amount.mean()),
        "amount_std": float(amount.std()),
        "genuine_amount_mean": float(amount[fraud == 0].mean()),
        "second_of_day_mean": float(sod.mean()),
        "second_of_day_std": float(sod.std()),
        "night_share": float(np.mean(sod // 3600 <= 6)),
        "terminals_used": int(len(np.unique(term))),
    }
    if scenario is not None:
        out["scenario_counts"] = {str(k): int((scenario == k).sum()) for k in (1, 2, 3)}
    return out


def main():
    import pandas as pd

    import refexec

    cache = "/tmp/fdx_ref_245d.pkl"
    if os.path.exists(cache):
        df = pd.read_pickle(cache)  # our own cache of the reference generator's output
    else:
        ns = refexec.load_namespace()
        c, t, df = ns["generate_dataset"](n_customers=5000, n_terminals=10000, nb_days=245,
                                          start_date="2024-06-01", r=5)
        df = ns["add_frauds"](c, t, df)
        df.to_pickle(cache)
    d = df[df.TX_TIME_DAYS < 183]
    s = stats_of(d.TX_TIME_DAYS.values.astype(np.int64), d.TX_TIME_SECONDS.values.astype(np.int64),
                 d.CUSTOMER_ID.values.astype(np.int64), d.TERMINAL_ID.values.astype(np.int64),
                 d.TX_AMOUNT.values.astype(np.float64), d.TX_FRAUD.values.astype(np.int64),
                 d.TX_FRAUD_SCENARIO.values.astype(np.int64), 5000, 183)
    s["source"] = ("reference generate_dataset(5000, 10000, nb_days=245, r=5) + add_frauds, first 183 days "
                   "(oracle/gen_synth_stats.py)")
    out = os.path.join(HERE, "..", "tests", "golden", "config1_stats.json")
    with open(out, "w") as f:
        json.dump(s, f, indent=1)
    print(json.dumps(s, indent=1))


if __name__ == "__main__":
    main()
