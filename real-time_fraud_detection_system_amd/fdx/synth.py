"""Fast synthetic transaction generators (bench / large-parity inputs; §8(f) row 3).

generate()         numpy, host arrays (CPU tests and small configs)
generate_device()  the same distributions generated on the GPU (csrc/fdx_synth.hip): the
                   host draws the customer profiles, the terminal map and the compromised
                   lists; the HIP kernels draw every transaction (Philox4x32-10), apply the
                   fraud scenarios and sort by time.  Config 4 (87.5M tx per rank) takes well
                   under a second instead of ~80 s on the host.

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
    scenario = np.zeros(len(secs), np.uint8)
    if frauds:
        fraud[amount > 220] = 1                                     # scenario 1
        scenario[amount > 220] = 1
        comp_t = np.zeros((nb_days + 1, n_terminals), bool)         # scenario 2
        comp_c = np.zeros((nb_days + 1, n_customers), bool)         # scenario 3
        for d in range(nb_days - 1):
            comp_t[d:d + 28, rng.choice(n_terminals, 2, replace=False)] = True
            comp_c[d:d + 14, rng.choice(n_customers, 3, replace=False)] = True
        s2 = comp_t[day, term]
        fraud[s2] = 1
        scenario[s2] = 2
        s3 = comp_c[day, cust] & (rng.random(len(cust)) < 1 / 3)
        amount[s3] = amount[s3] * 5
        fraud[s3] = 1
        scenario[s3] = 3
    return {
        "ts": START_NS + secs.astype(np.int64) * NS,
        "customer": (cust + customer_offset).astype(np.int32),
        "terminal": term.astype(np.int32),
        "amount": amount.astype(np.float64),
        "fraud": fraud,
        "scenario": scenario,
        "day": day.astype(np.int32),
        "tid": np.arange(len(secs), dtype=np.int64),
    }


def _profiles(n_customers, n_terminals, r, seed, terminal_seed):
    """Customer profiles and the terminal map, drawn exactly as generate() draws them."""
    rng = np.random.default_rng(seed)
    cx, cy = rng.uniform(0, 100, n_customers), rng.uniform(0, 100, n_customers)
    mean_amount = rng.uniform(5, 100, n_customers)
    mean_nb = rng.uniform(0, 4, n_customers)
    trng = np.random.default_rng(terminal_seed)  # shared by all ranks: one terminal map
    tx, ty = trng.uniform(0, 100, n_terminals), trng.uniform(0, 100, n_terminals)
    return rng, cx, cy, mean_amount, mean_nb, tx, ty


def generate_device(n_customers=5000, n_terminals=10000, nb_days=183, r=5.0, seed=0, customer_offset=0,
                    frauds=True, terminal_seed=10_000, device=None, with_scenario=False, stream=None,
                    n_customers_total=None):
    """generate() on the GPU: a dict of device tensors in global time order --
    ts int64 ns, customer int32 (+ customer_offset), terminal int32, amount float64, fraud uint8
    (and scenario uint8, day int32 when with_scenario).

    The rows of customers [customer_offset, customer_offset + n_customers) of a population of
    n_customers_total (default: customer_offset + n_customers): the profiles and the compromised
    customers are drawn for the whole population and every transaction draw is keyed by the
    global customer id, so a range's output is the population's generation filtered to its
    customers, row for row -- the union over any split of the ids is the same data (the
    multi-GPU bench's like-for-like 1 -> N curve)."""
    import ctypes

    import torch

    from . import _lib, ops
    from ._lib import check

    dev = device or ops.require_gpu()
    c0, n_customers = int(customer_offset), int(n_customers)
    n_pop = c0 + n_customers if n_customers_total is None else int(n_customers_total)
    if not (0 <= c0 and c0 + n_customers <= n_pop < 2**31):
        raise ValueError(f"customers [{c0}, {c0 + n_customers}) outside the population [0, {n_pop})")
    rng, cx, cy, mean_amount, mean_nb, tx, ty = _profiles(n_pop, n_terminals, r, seed, terminal_seed)
    cx, cy, mean_amount, mean_nb = (a[c0:c0 + n_customers] for a in (cx, cy, mean_amount, mean_nb))
    sampler = _TerminalSampler(tx, ty, r)
    lo, hi = sampler.ranges(cx, cy)
    frng = np.random.default_rng([seed, 7919])
    ct, cc = [], []
    if frauds:  # add_frauds: for day in range(max day): 2 terminals for 28 days, 3 customers for 14
        for d in range(nb_days - 1):
            ct += [(int(t), d) for t in frng.choice(n_terminals, 2, replace=False)]
            cc += [(int(c) - c0, d) for c in frng.choice(n_pop, 3, replace=False) if c0 <= c < c0 + n_customers]
    comp_t = np.array(sorted(ct), np.int32).reshape(-1, 2)
    comp_c = np.array(sorted(cc), np.int32).reshape(-1, 2)

    def D(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)

    keep = dict(cx=D(cx, torch.float64), cy=D(cy, torch.float64), ma=D(mean_amount, torch.float64),
                mn=D(mean_nb, torch.float64), xs=D(sampler.xs, torch.float64), ys=D(sampler.ys, torch.float64),
                order=D(sampler.order, torch.int32), lo=D(lo, torch.int32), hi=D(hi, torch.int32),
                ct=D(comp_t if len(comp_t) else np.zeros((1, 2), np.int32), torch.int32),
                cc=D(comp_c if len(comp_c) else np.zeros((1, 2), np.int32), torch.int32))
    p = lambda t: t.data_ptr()  # noqa: E731
    desc = _lib.SynthDesc(int(n_customers), int(n_terminals), int(nb_days), float(r),
                          int(np.random.default_rng([seed, 104729]).integers(0, 2**63)),
                          p(keep["cx"]), p(keep["cy"]), p(keep["ma"]), p(keep["mn"]), p(keep["xs"]), p(keep["ys"]),
                          p(keep["order"]), p(keep["lo"]), p(keep["hi"]), p(keep["ct"]), len(comp_t),
                          p(keep["cc"]), len(comp_c), int(START_NS), int(customer_offset))
    L = _lib.load()
    ws = ops.workspace(L.fdx_synth_workspace_size(ctypes.byref(desc), 0), dev)
    n_tx = ctypes.c_int64()
    check(L.fdx_synth_plan(ctypes.byref(desc), ops._ptr(ws), ws.numel(), ctypes.byref(n_tx), ops._s(stream)),
          "fdx_synth_plan")
    n = n_tx.value
    need = L.fdx_synth_workspace_size(ctypes.byref(desc), n)
    if need > ws.numel():  # the plan's offsets sit at the front of the larger workspace
        ws2 = ops.workspace(need, dev)
        ws2[: ws.numel()].copy_(ws)
        ws = ws2
    out = {"ts": torch.empty(n, dtype=torch.int64, device=dev), "customer": torch.empty(n, dtype=torch.int32, device=dev),
           "terminal": torch.empty(n, dtype=torch.int32, device=dev),
           "amount": torch.empty(n, dtype=torch.float64, device=dev),
           "fraud": torch.empty(n, dtype=torch.uint8, device=dev)}
    if with_scenario:
        out["scenario"] = torch.empty(n, dtype=torch.uint8, device=dev)
        out["day"] = torch.empty(n, dtype=torch.int32, device=dev)
    check(L.fdx_synth_fill(ctypes.byref(desc), n, ops._ptr(ws), ws.numel(), *[ops._ptr(out[k]) for k in
                                                                               ("ts", "customer", "terminal", "amount",
                                                                                "fraud")],
                           ops._ptr(out.get("scenario")), ops._ptr(out.get("day")), ops._s(stream)), "fdx_synth_fill")
    torch.cuda.current_stream(dev).synchronize()  # keep the host-side inputs alive until the kernels ran
    del keep
    return out
