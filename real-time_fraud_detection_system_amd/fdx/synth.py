"""Fast synthetic transaction generator (bench / large-parity inputs; not the product).

Same distributions as the reference handbook generator
(fraud_detection_model/data_generator.ipynb: customer profiles :113-140, terminal profiles
:285-303, terminals within radius r :420-437, daily Poisson transactions with Gaussian
time-of-day and amount :786-834, global time sort + TRANSACTION_ID :1339-1371, and the three
fraud scenarios of add_frauds :1732-1782), vectorised with numpy.  It does NOT reproduce the
reference's RNG stream (that one is pure Python, ~100 s per 1.75M rows); exact parity on
the reference's own data is pinned by tests/golden/ instead.
"""
from __future__ import annotations

import numpy as np

START_NS = np.datetime64("2024-06-01T00:00:00", "ns").astype(np.int64)
NS = 1_000_000_000


class _TerminalSampler:
    """Uniform choice among the terminals within radius r of a customer
    (get_list_terminals_within_radius + random.choice, data_generator.ipynb:420-437, :821)
    without materialising the per-customer lists: draw uniformly from the terminals whose x
    lies in [cx - r, cx + r] (a contiguous range of the x-sorted terminals) and reject the
    draws outside the disk.  Exact in distribution; scales to millions of terminals."""

    def __init__(self, tx, ty, r):
        self.order = np.argsort(tx, kind="stable")
        self.xs, self.ys = tx[self.order], ty[self.order]
        self.r = r

    def count(self, cx, cy):
        from scipy.spatial import cKDTree

        tree = cKDTree(np.stack([self.xs, self.ys], axis=1))
        return tree.query_ball_point(np.stack([cx, cy], axis=1), r=self.r - 1e-12, return_length=True,
                                     workers=-1)

    def sample(self, rng, px, py):
        lo = np.searchsorted(self.xs, px - self.r, side="left")
        hi = np.searchsorted(self.xs, px + self.r, side="right")
        out = np.full(len(px), -1, np.int64)
        pending = np.arange(len(px))
        while len(pending):
            span = hi[pending] - lo[pending]
            cand = lo[pending] + (rng.random(len(pending)) * span).astype(np.int64)
            dx, dy = self.xs[cand] - px[pending], self.ys[cand] - py[pending]
            ok = np.sqrt(dx * dx + dy * dy) < self.r
            out[pending[ok]] = self.order[cand[ok]]
            pending = pending[~ok]
        return out


def generate(n_customers=5000, n_terminals=10000, nb_days=183, r=5.0, seed=0, customer_offset=0,
             frauds=True, terminal_seed=10_000):
    """Returns a dict of numpy arrays in global time order:
    ts (int64 ns), customer (int32), terminal (int32), amount (f64), fraud (u8), tid (int64)."""
    rng = np.random.default_rng(seed)
    cx, cy = rng.uniform(0, 100, n_customers), rng.uniform(0, 100, n_customers)
    mean_amount = rng.uniform(5, 100, n_customers)
    std_amount = mean_amount / 2
    mean_nb = rng.uniform(0, 4, n_customers)
    trng = np.random.default_rng(terminal_seed)  # shared by all ranks: one terminal map
    tx, ty = trng.uniform(0, 100, n_terminals), trng.uniform(0, 100, n_terminals)
    sampler = _TerminalSampler(tx, ty, r)
    has_term = sampler.count(cx, cy) > 0

    counts = rng.poisson(np.broadcast_to(mean_nb, (nb_days, n_customers)))  # [day, customer]
    day_idx, cust_idx = np.nonzero(counts)
    reps = counts[day_idx, cust_idx]
    day = np.repeat(day_idx, reps)
    cust = np.repeat(cust_idx, reps)
    t = rng.normal(86400 / 2, 20000, size=len(day)).astype(np.int64)
    amount = rng.normal(mean_amount[cust], std_amount[cust])
    neg = amount < 0
    amount[neg] = rng.uniform(0, mean_amount[cust[neg]] * 2)
    amount = np.round(amount, 2)
    keep = (t > 0) & (t < 86400) & has_term[cust]
    day, cust, t, amount = day[keep], cust[keep], t[keep], amount[keep]
    term = sampler.sample(rng, cx[cust], cy[cust])
    secs = t + day * 86400
    order = np.argsort(secs, kind="stable")
    secs, day, cust, term, amount = secs[order], day[order], cust[order], term[order], amount[order]

    fraud = np.zeros(len(secs), np.uint8)
    if frauds:
        fraud[amount > 220] = 1                                     # scenario 1
        comp_t = np.zeros((nb_days + 1, n_terminals), bool)         # scenario 2
        comp_c = np.zeros((nb_days + 1, n_customers), bool)         # scenario 3
        for d in range(nb_days - 1):
            comp_t[d:d + 28, rng.choice(n_terminals, 2, replace=False)] = True
            comp_c[d:d + 14, rng.choice(n_customers, 3, replace=False)] = True
        fraud[comp_t[day, term]] = 1
        s3 = comp_c[day, cust] & (rng.random(len(cust)) < 1 / 3)
        amount[s3] = amount[s3] * 5
        fraud[s3] = 1
    return {
        "ts": START_NS + secs.astype(np.int64) * NS,
        "customer": (cust + customer_offset).astype(np.int32),
        "terminal": term.astype(np.int32),
        "amount": amount.astype(np.float64),
        "fraud": fraud,
        "tid": np.arange(len(secs), dtype=np.int64),
    }
