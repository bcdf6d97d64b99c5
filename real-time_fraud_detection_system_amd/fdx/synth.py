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
    without materialising the per-customer lists: terminals are sorted by (y band of height r,
    x); the disk around a customer lies inside three bands, and in each band its x-range
    [cx - r, cx + r] is one contiguous run.  Draw uniformly from the union of the three runs
    and reject the draws outside the disk (acceptance ~ pi/6).  Exact in distribution; scales
    to millions of terminals."""

    def __init__(self, tx, ty, r):
        self.r = float(r)
        band = np.floor(ty / self.r).astype(np.int64)
        self.order = np.lexsort((tx, band))
        self.xs, self.ys = tx[self.order], ty[self.order]
        self.key = band[self.order] * 1000.0 + self.xs       # x < 1000: sorted by (band, x)
        self.n_bands = int(band.max()) + 1 if len(band) else 0

    def has_terminal(self, cx, cy):
        from scipy.spatial import cKDTree

        tree = cKDTree(np.stack([self.xs, self.ys], axis=1))
        d, _ = tree.query(np.stack([cx, cy], axis=1), k=1, distance_upper_bound=self.r, workers=-1)
        return d < self.r

    def ranges(self, px, py):
        """[n, 3] lo / hi index runs of the three bands around each point"""
        b = np.floor(py / self.r).astype(np.int64)
        lo = np.empty((len(px), 3), np.int64)
        hi = np.empty((len(px), 3), np.int64)
        for k in range(3):
            bk = b - 1 + k
            ok = (bk >= 0) & (bk < self.n_bands)
            base = bk * 1000.0
            lo[:, k] = np.searchsorted(self.key, base + px - self.r, side="left")
            hi[:, k] = np.where(ok, np.searchsorted(self.key, base + px + self.r, side="right"), lo[:, k])
        return lo, hi

    def sample(self, rng, px, py, lo, hi):
        """one terminal per point; lo / hi: ranges() of each point"""
        span = hi - lo
        c1 = span[:, 0]
        c2 = c1 + span[:, 1]
        tot = c2 + span[:, 2]
        out = np.full(len(px), -1, np.int64)
        pending = np.flatnonzero(tot > 0)
        while len(pending):
            u = (rng.random(len(pending)) * tot[pending]).astype(np.int64)
            a, b = c1[pending], c2[pending]
            k = (u >= a).astype(np.int64) + (u >= b)
            off = u - np.where(k == 0, 0, np.where(k == 1, a, b))
            cand = lo[pending, k] + off
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
    has_term = sampler.has_terminal(cx, cy)
    lo_c, hi_c = sampler.ranges(cx, cy)

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
    term = sampler.sample(rng, cx[cust], cy[cust], lo_c[cust], hi_c[cust])
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
