"""LDS-cycle model of k_forest_rank's node reads for different row orders (host only).

Per walk step every wave issues one ds_read_b32 of its lanes' nodes; the LDS serves lanes
0-31 and 32-63 in one cycle each when conflict-free, and each extra DISTINCT address on a
busy bank (bank = word address mod 32) adds a cycle (MI355X_MICROARCH.md §LDS).  This
counts those cycles for the depth-20 bench forest over a sample of bench-like rows, for the
row orders given, so a reordering of the scoring rows can be judged before it is built.

usage: python tools/lds_sim.py [n_customers] [trees]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "real-time_fraud_detection_system_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]


def rows(n_customers):
    import oracle
    from fdx import synth

    d = synth.generate(n_customers, 2 * n_customers, 183, seed=1234)
    f = oracle.featurize_arrays(d["ts"], d["customer"], d["terminal"], d["amount"], d["fraud"])
    names = ["TX_DURING_WEEKEND", "TX_DURING_NIGHT"] + oracle.CUSTOMER_COLS + oracle.TERMINAL_COLS
    X = np.column_stack([d["amount"]] + [f[k] for k in names])
    return X, d


def ranks(R, z32):
    n = z32.shape[0]
    xv = np.zeros((n, 16), np.int64)
    for f in range(15):
        u = R["thr"][R["thr_off"][f]:R["thr_off"][f + 1]]
        xv[:, f] = np.searchsorted(u, z32[:, f], side="left") << 16
    xv[:, 15] = 0x4000 << 16
    return xv


def cycles(R, xv, trees):
    """node-read LDS cycles per 64-row wave-step, summed over the given trees, and
    the conflict-free count (2 per wave-step)."""
    nodes = R["nodes"].astype(np.int64)
    n = xv.shape[0] - xv.shape[0] % 64
    xv = xv[:n]
    g = np.arange(n) // 32
    tot = 0
    steps = 0
    rows_ = np.arange(n)
    for t in trees:
        p = np.full(n, R["root"][t], np.int64)
        for _ in range(int(R["depth"][t])):
            nd = nodes[p]
            f = (nd >> 12) & 15
            d = xv[rows_, f] - nd
            st = np.clip(d, 1, None)
            st = np.minimum(st, nd & 0xFFF)
            st = np.where(d <= 0, 1, st)
            st = np.where((nd & 0xFFF) == 0, 0, st)
            p = p + st
            # distinct addresses per (group, bank); cycles of a group = max over banks
            key = np.unique(g * (1 << 32) + p)
            gk, bk = key >> 32, (key & 0xFFFFFFFF) % 32
            cnt = np.bincount(gk * 32 + bk, minlength=(n // 32) * 32).reshape(-1, 32)
            tot += int(cnt.max(axis=1).sum())
            steps += 1
    return tot / (n // 64) / steps, steps


def main():
    from test_rank_layout import pack_rank

    nc = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    nt = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    R = pack_rank(z)
    t0 = time.time()
    X, d = rows(nc)
    z32 = ((X - z["mean"]) / z["scale"]).astype(np.float32)
    xv = ranks(R, z32)
    print(f"{len(X)} rows featurized in {time.time() - t0:.1f} s", flush=True)
    trees = list(range(0, 100, 100 // nt))[:nt]
    rng = np.random.default_rng(0)
    cperm = np.lexsort((np.arange(len(X)), d["customer"]))
    # the interleaved layout: 21 customers per group, slot = step * 21 + lane
    orders = {"time": np.arange(len(X)), "customer": cperm, "random": rng.permutation(len(X))}
    # leaf of tree 0 / lexicographic leaves of trees 0..k as sort keys
    nodes = R["nodes"].astype(np.int64)

    def leaf(t):
        n = len(X)
        p = np.full(n, R["root"][t], np.int64)
        for _ in range(int(R["depth"][t])):
            nd = nodes[p]
            dd = xv[np.arange(n), (nd >> 12) & 15] - nd
            st = np.where(dd <= 0, 1, np.minimum(np.clip(dd, 1, None), nd & 0xFFF))
            p = p + np.where((nd & 0xFFF) == 0, 0, st)
        return p

    l0, l1 = leaf(1), leaf(2)
    orders["leaf_t1"] = np.lexsort((np.arange(len(X)), l0))
    orders["leaf_t1_t2"] = np.lexsort((l1, l0))
    orders["lex_ranks"] = np.lexsort(tuple(xv[:, f] for f in range(14, -1, -1)))
    imp = np.argsort(-np.bincount((nodes[R["orig"] >= 0] >> 12) & 15, minlength=16)[:15])
    orders["lex_by_use"] = np.lexsort(tuple(xv[:, f] for f in imp[::-1]))
    for name, o in orders.items():
        c, s = cycles(R, xv[o], trees)
        print(f"{name:12s} node-read cycles/wave-step {c:.2f} (conflict-free 2.00) over {s} steps", flush=True)


if __name__ == "__main__":
    main()
