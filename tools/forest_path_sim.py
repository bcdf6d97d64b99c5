"""Walk-step model of the forest traversal: how many node steps a wave executes per row,
wave-paced (k_forest_rank: every lane waits for the wave's deepest chain) vs lane-paced
(k_forest_lanes: a lane moves to its next row when its own chains are at leaves, the move
gated on >= TH finished lanes), from the bench model's true path lengths on its check rows.

    python tools/forest_path_sim.py [bench_assets/rf100_d20.npz]

Paths are computed with sklearn's float64 <= rule on the scaled check rows (the same leaves
the GPU kernels reach); chunks = 18 equal tree ranges (the bench forest's LDS chunks hold ~6
trees); 64 lanes x 68 rows per lane (17.76M rows over 256 blocks x 1,024 lanes).

Result (bench model): mean path 19.76 of 20 steps, so the wave-paced walk already executes
~1.0x the steps the rows need and lane pacing has nothing to recover.
"""
import sys

import numpy as np


def path_lengths(z):
    off, L, R, F, T = z["node_offsets"], z["left"], z["right"], z["feature"], z["threshold"]
    X = (z["check_X"] - z["mean"]) / z["scale"]  # check rows are unscaled; thresholds are on scaled features
    n, nt = len(X), len(off) - 1
    P = np.zeros((n, nt), np.int32)
    rows = np.arange(n)
    for t in range(nt):
        node = np.zeros(n, np.int64)
        while True:
            g = off[t] + node
            internal = L[g] != -1
            if not internal.any():
                break
            f = np.where(internal, F[g], 0).astype(np.int64)
            go = np.where(X[rows, f] <= T[g], L[g], R[g])
            node = np.where(internal, go, node)
            P[:, t] += internal
    return P


def simulate(P, E, TH, chunks=18, lanes=64, rows_per_lane=68, seed=1):
    """-> (steps per row, advance blocks per row) for exit tests every E steps."""
    rng = np.random.default_rng(seed)
    bounds = np.linspace(0, P.shape[1], chunks + 1).astype(int)
    steps = blocks = rows = 0
    for c in range(0, chunks, 2):
        a, b = bounds[c], bounds[c + 1]
        need = np.maximum(P[rng.integers(0, len(P), (lanes, rows_per_lane))][:, :, a:b].max(axis=2), 1)
        ptr = np.zeros(lanes, int)
        rem = need[:, 0].copy()
        t = nb = 0
        while (ptr < rows_per_lane).any():
            t += E
            act = ptr < rows_per_lane
            rem[act] -= E
            done = act & (rem <= 0)
            if done.sum() >= min(TH, act.sum()):
                nb += 1
                for lane in np.nonzero(done)[0]:
                    ptr[lane] += 1
                    if ptr[lane] < rows_per_lane:
                        rem[lane] = need[lane, ptr[lane]]
        steps += t
        blocks += nb
        rows += rows_per_lane
    return steps / rows, blocks / rows


def main():
    z = np.load(sys.argv[1] if len(sys.argv) > 1 else "bench_assets/rf100_d20.npz")
    P = path_lengths(z)
    print(f"path length: mean {P.mean():.2f}, median {np.median(P):.0f}, max {P.max()}")
    for E in (2, 4):
        for TH in (1, 8, 16, 24, 32, 64):
            s, b = simulate(P, E, TH)
            kind = "wave-paced" if TH == 64 else "lane-paced"
            print(f"E={E} TH={TH:2d} ({kind}): {s:5.2f} steps/row, {b:4.2f} advances/row")


if __name__ == "__main__":
    main()
