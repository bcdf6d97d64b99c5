"""Random sklearn-layout forests for the forest tests (host only, no GPU)."""
import numpy as np


def random_forest(rng, n_trees, depth, n_feat=15, p_leaf=0.15):
    """Random sklearn-layout trees (pre-order, -1 leaves) for chunking / global-path tests."""
    L, R, F, TH, ML, V, off = [], [], [], [], [], [], [0]
    for _ in range(n_trees):
        left, right, feat, thr, ml, val = [], [], [], [], [], []

        def build(d):
            i = len(left)
            left.append(-1); right.append(-1); feat.append(-2); thr.append(-2.0); ml.append(0)
            val.append(float(rng.integers(0, 1000)) / 999.0)
            if d < depth and (d < 2 or rng.random() > p_leaf):
                feat[i] = int(rng.integers(0, n_feat)); thr[i] = float(rng.normal()) * 1.3
                ml[i] = int(rng.random() < 0.5)
                left[i] = build(d + 1)
                right[i] = build(d + 1)
            return i

        build(0)
        L += left; R += right; F += feat; TH += thr; ML += ml; V += val
        off.append(off[-1] + len(left))
    return dict(left=np.array(L, np.int64), right=np.array(R, np.int64), feature=np.array(F, np.int64),
                threshold=np.array(TH), missing_left=np.array(ML, np.uint8), value1=np.array(V),
                node_offsets=np.array(off, np.int64))
