"""Forest chunks that are one walk group (<= 8 trees, every chunk of the bench forest): the tile
loop folds a tile's leaf values one tile late and loads its output slots with its rank rows
(k_forest_rank, one_group).  Probabilities must equal sklearn's (golden fixtures, the bench
model's check rows), the C oracle's and the wide-layout kernel's bit for bit -- chunks of 1..8
trees, several tiles per block (n past 256 x 1,024 rows), a ragged last tile, NaN rows (the
missing_go_to_left walk) and the scoring-slot scatter of the fused path.
Reference call: pyspark/scripts/fraud_detection.py:190-193 (predict_proba of the loaded model).
"""
import os

import numpy as np
import pytest
import torch

import oracle
from fdx import ops
from fdx._lib import FdxError
from forest_gen import random_forest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = [1, 2, 3, 4, 5]  # v1 (10 chains per lane, interleaved pairs), v2 (6), compact v2 (6), v2 (10), paired v2


def T(a, dt, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)


def _arrays(z):
    return {k: z[k].astype(np.int64) if k in ("left", "right", "feature") else z[k]
            for k in ("node_offsets", "left", "right", "feature", "threshold", "missing_left", "value1")}


def _set(f, v):
    try:
        f.set_variant(v)
    except FdxError:  # the variant's node format does not hold this forest
        return False
    return True


@pytest.mark.parametrize("variant", VARIANTS)
def test_one_group_golden_fixtures(dev, golden, variant):
    """sklearn's own probabilities (3- and 5-tree fixtures: one chunk), ~700k rows."""
    for name in ("forest_rf3.npz", "forest_rf5d8.npz"):
        z = golden(name)
        f = ops.Forest(_arrays(z), 15, z["mean"], z["scale"])
        if not _set(f, variant):
            continue
        reps = -(-700_001 // len(z["X"]))
        X = np.vstack([z["X"]] * reps)
        p = f.predict(T(X, torch.float64, dev)).cpu().numpy()
        np.testing.assert_array_equal(p, np.concatenate([z["proba"]] * reps), err_msg=name)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("n_trees,depth", [(1, 12), (2, 9), (4, 10), (6, 11), (7, 11), (8, 10), (20, 12)])
def test_one_group_random_forests_vs_oracle(dev, variant, n_trees, depth):
    """Forests whose chunks hold 1..8 trees (20 deep trees: several chunks, the running sum
    across launches), then the same rows with NaNs; n not a multiple of the tile."""
    rng = np.random.default_rng(1000 * n_trees + depth)
    arr = random_forest(rng, n_trees, depth, p_leaf=0.05)
    f = ops.Forest(arr, 15)
    if not _set(f, variant):
        pytest.skip("node format does not hold this forest")
    g = ops.Forest(arr, 15)
    g.set_variant(0)  # the wide-layout kernel as the GPU reference
    n = 700_001 + n_trees
    X = rng.normal(size=(n, 15))
    Xd = T(X, torch.float64, dev)
    p = f.predict(Xd).cpu().numpy()
    np.testing.assert_array_equal(p, g.predict(Xd).cpu().numpy())
    sel = rng.choice(n, 20_000, replace=False)
    np.testing.assert_array_equal(p[sel], oracle.forest_predict(X[sel], arr))
    Xn = X.copy()
    Xn[rng.random(Xn.shape) < 0.03] = np.nan
    pn = f.predict(T(Xn, torch.float64, dev)).cpu().numpy()
    np.testing.assert_array_equal(pn[sel], oracle.forest_predict(Xn[sel], arr))


def test_one_group_bench_model(dev):
    """The bench RF(100, depth 20), 18 chunks of 3-6 trees: 700k rows == the wide layout and the
    oracle (sampled); the check rows == sklearn."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arr = _arrays(z)
    f = ops.Forest(arr, 15, z["mean"], z["scale"])
    assert f.n_chunks > 1
    g = ops.Forest(arr, 15, z["mean"], z["scale"])
    g.set_variant(0)
    rng = np.random.default_rng(5)
    X = np.vstack([z["check_X"]] * 171)
    X = X * (1 + rng.normal(scale=0.05, size=X.shape) * (rng.random(X.shape) < 0.5))
    Xd = T(X, torch.float64, dev)
    p = f.predict(Xd).cpu().numpy()
    np.testing.assert_array_equal(p, g.predict(Xd).cpu().numpy())
    sel = rng.choice(len(X), 20_000, replace=False)
    np.testing.assert_array_equal(p[sel], oracle.forest_predict(X[sel], arr, z["mean"], z["scale"]))
    pc = f.predict(T(np.vstack([z["check_X"]] * 64), torch.float64, dev)).cpu().numpy()
    np.testing.assert_array_equal(pc, np.concatenate([z["check_proba"]] * 64))


def test_one_launch_chunk_loop(dev):
    """Every chunk of the bench forest is one walk group, so a large batch walks all 18 chunks in
    ONE k_forest_rank launch (the kernel's chunk loop, running sums handed between chunks by the
    lane that owns the row); with leaf ids it is one launch per chunk, and a small batch runs every
    chunk at once.  All three give the same probabilities, bit for bit, and the leaf ids are the
    oracle's."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arr = _arrays(z)
    f = ops.Forest(arr, 15, z["mean"], z["scale"])
    n = 300_017  # > 256 CUs x 1,024 rows: past the all-chunks-at-once size
    assert f.n_chunks == 18
    assert f.traverse_launches(n) == 1
    assert f.traverse_launches(n, want_leaves=True) == f.n_chunks
    assert f.traverse_launches(1000) == 1 and f.traverse_launches(0) == 0
    rng = np.random.default_rng(11)
    X = np.vstack([z["check_X"]] * (n // len(z["check_X"]) + 1))[:n]
    X = X * (1 + rng.normal(scale=0.05, size=X.shape) * (rng.random(X.shape) < 0.5))
    Xd = T(X, torch.float64, dev)
    p1 = f.predict(Xd).cpu().numpy()
    pl, leaves = f.predict(Xd, want_leaves=True)
    np.testing.assert_array_equal(p1, pl.cpu().numpy())
    ps = f.predict(Xd[:1000]).cpu().numpy()
    np.testing.assert_array_equal(ps, p1[:1000])
    sel = rng.choice(n, 5_000, replace=False)
    np.testing.assert_array_equal(p1[sel], oracle.forest_predict(X[sel], arr, z["mean"], z["scale"]))
    _, want_leaves = oracle.forest_predict(X[sel[:200]], arr, z["mean"], z["scale"], want_leaves=True)
    np.testing.assert_array_equal(leaves.cpu().numpy()[sel[:200]], want_leaves)


@pytest.mark.parametrize("variant", [0] + VARIANTS)
def test_traverse_launch_count(dev, variant):
    """fdx_forest_traverse_launches per layout: the wide layout launches once per chunk; a rank
    layout walks every chunk in one launch when each is one walk group (else one per chunk), per
    32-bit row range (128M rows of 32-B rank rows, 64M of 64-B v2 rows); one per chunk with leaf
    ids; small batches run every chunk at once.  20 trees of depth 12: several chunks."""
    rng = np.random.default_rng(77)
    arr = random_forest(rng, 20, 12, p_leaf=0.05)
    f = ops.Forest(arr, 15)
    if not _set(f, variant):
        pytest.skip("node format does not hold this forest")
    nc = f.n_chunks
    assert nc > 1
    big = 3_000_000
    assert f.traverse_launches(0) == 0
    if variant == 0:
        assert f.traverse_launches(big) == nc
        return
    k = f.traverse_launches(big)
    assert k in (1, nc)
    rows = (2**32 - 1) // (64 if variant in (2, 4, 5) else 32) // 1024 * 1024
    assert f.traverse_launches(rows) == k
    assert f.traverse_launches(rows + 1) == 2 * k
    assert f.traverse_launches(big, want_leaves=True) == nc
    assert f.traverse_launches(1000) == 1


def test_row_ranges_past_32_bit_offsets(dev):
    """A batch larger than one 32-bit-addressable row range (134,216,704 rows of 32-B rank rows:
    the one-group tile loop's byte offsets) is walked range by range, each launch over base
    pointers moved to its range.  Rows on both sides of the boundary == the oracle; with the
    output permutation (absolute output slots) every row lands where the plain traversal puts it."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arr = _arrays(z)
    f = ops.Forest(arr, 15, z["mean"], z["scale"])
    rr = 134_216_704
    n = rr + 3001
    assert f.traverse_launches(n) == 2 and f.traverse_launches(rr) == 1
    chk = T(z["check_X"], torch.float64, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(21)
    pick = torch.randint(0, chk.shape[0], (n,), device=dev, generator=g)
    Xd = chk[pick]
    del pick
    p = f.predict(Xd)
    rng = np.random.default_rng(21)
    idx = np.concatenate([np.arange(rr - 2000, n), rng.choice(rr - 2000, 3000, replace=False)])
    X = Xd[torch.from_numpy(idx).to(dev)].cpu().numpy()
    np.testing.assert_array_equal(p[torch.from_numpy(idx).to(dev)].cpu().numpy(),
                                  oracle.forest_predict(X, arr, z["mean"], z["scale"]))
    ws = torch.empty(f.workspace_size(n), dtype=torch.uint8, device=dev)
    ops.forest_prepare(f, Xd, ws)
    del Xd
    perm = torch.randperm(n, device=dev, generator=g).to(torch.int32)
    out = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    ops.forest_traverse_perm(f, n, ws, out, perm)
    assert torch.equal(out[perm.long()], p)


def test_prepare_row_major_spans(dev):
    """fdx_forest_prepare of dense row-major X stages each wave's 64 rows as one contiguous span
    (k_prepare_rows): a ragged last span, NaN rows, an X that starts 8 bytes off a 16-byte
    boundary (a view from row 1) and a padded row stride (the per-lane kernel) all give the
    oracle's probabilities."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arr = _arrays(z)
    f = ops.Forest(arr, 15, z["mean"], z["scale"])
    rng = np.random.default_rng(31)
    n = 64 * 4099 + 37
    X = np.vstack([z["check_X"]] * (n // len(z["check_X"]) + 2))[:n + 1]
    X = X * (1 + rng.normal(scale=0.05, size=X.shape) * (rng.random(X.shape) < 0.5))
    X[rng.random(X.shape) < 0.002] = np.nan
    sel = np.concatenate([np.arange(0, 200), np.arange(n - 200, n), rng.choice(n, 3000, replace=False)])
    want = oracle.forest_predict(X[1:][sel], arr, z["mean"], z["scale"])
    Xall = T(X, torch.float64, dev)
    p_view = f.predict(Xall[1:]).cpu().numpy()  # 120 B past the allocation: 8-B aligned
    p_dense = f.predict(Xall[1:].contiguous()).cpu().numpy()
    pad = torch.zeros((n, 16), dtype=torch.float64, device=dev)
    pad[:, :15] = Xall[1:]
    p_pad = f.predict(pad[:, :15]).cpu().numpy()
    np.testing.assert_array_equal(p_dense[sel], want)
    np.testing.assert_array_equal(p_view, p_dense)
    np.testing.assert_array_equal(p_pad, p_dense)


def test_refused_variant_leaves_the_forest_intact(dev):
    """a refused set_variant must leave the forest as it was.  The deployed model
    (rank layout v2, 22 threshold slots; default variant 5, paired planes) cannot run v1 (a feature has 96k thresholds: the v1
    rebuild fails after the v2 buffers were freed) nor compact v2 (more slots than features);
    after each refusal the forest is back in v2 with its variant and chunks, and predict is
    still sklearn's on the notebook's test rows."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf_deployed.npz"))
    f = ops.Forest(_arrays(z), 15, z["mean"], z["scale"])
    v0, nc0 = f.variant, f.n_chunks
    assert v0 == 5  # paired planes: every tree fits below its 22 slot planes
    X = T(z["test_X"][:20_000], torch.float64, dev)
    want = z["test_proba1"][:20_000]
    for bad in (1, 3, 1):
        with pytest.raises(FdxError):
            f.set_variant(bad)
        assert f.variant == v0
        np.testing.assert_array_equal(f.predict(X).cpu().numpy(), want)
    f.set_variant(4)
    np.testing.assert_array_equal(f.predict(X).cpu().numpy(), want)
    f.set_variant(5)  # paired planes: 22 slots at the top of the LDS, every tree below them
    np.testing.assert_array_equal(f.predict(X).cpu().numpy(), want)
    Xn = z["test_X"][:20_000].copy()
    Xn[np.random.default_rng(3).random(Xn.shape) < 0.02] = np.nan
    f.set_variant(2)
    pn2 = f.predict(T(Xn, torch.float64, dev)).cpu().numpy()
    f.set_variant(5)
    np.testing.assert_array_equal(f.predict(T(Xn, torch.float64, dev)).cpu().numpy(), pn2)
    assert f.n_chunks == nc0
    np.testing.assert_array_equal(f.predict(X).cpu().numpy(), want)


def _lone_and_stump():
    lone = dict(left=np.array([-1]), right=np.array([-1]), feature=np.array([-2]), threshold=np.array([-2.0]),
                missing_left=np.array([0], np.uint8), value1=np.array([0.375]))
    stump = dict(left=np.array([1, -1, -1]), right=np.array([2, -1, -1]), feature=np.array([3, -2, -2]),
                 threshold=np.array([0.25, -2.0, -2.0]), missing_left=np.array([1, 0, 0], np.uint8),
                 value1=np.array([0.0, 0.125, 0.875]))
    return lone, stump


def _forest_of(parts):
    b = {k: np.concatenate([pt[k] for pt in parts]) for k in parts[0]}
    b["node_offsets"] = np.concatenate([[0], np.cumsum([len(pt["left"]) for pt in parts])]).astype(np.int64)
    for k in ("left", "right", "feature"):
        b[k] = b[k].astype(np.int64)
    return b


@pytest.mark.parametrize("kinds", ["lone", "stump", "lone+stump", "stump+lone+stump"])
def test_one_group_degenerate_depths(dev, kinds):
    """Chunks whose deepest tree has depth 0 (a single leaf) or 1 (a stump): the walk's first step
    from the launch-uniform root words and its read-free last step coincide or vanish.  Every
    row == the C oracle, NaN rows included (missing_go_to_left of the stump)."""
    lone, stump = _lone_and_stump()
    arr = _forest_of([{"lone": lone, "stump": stump}[k] for k in kinds.split("+")])
    f = ops.Forest(arr, 15)
    assert f.variant == 1
    rng = np.random.default_rng(len(kinds))
    X = rng.normal(size=(300_001, 15))
    X[rng.random(X.shape) < 0.03] = np.nan
    for Xi in (np.nan_to_num(X, nan=0.5), X):
        p = f.predict(T(Xi, torch.float64, dev)).cpu().numpy()
        np.testing.assert_array_equal(p, oracle.forest_predict(Xi, arr))


def test_prepare_integer_and_ratio_shortcuts(dev):
    """fdx_forest_prepare (k_prepare_st) ranks a small non-negative integer through the integer
    table and a value that is exactly fr / nb (nb = the previous column, a small integer) through
    the ratio table -- the terminal counts and risks of the reference's layout.  Both must equal
    the search bit for bit: the bench model's check rows, the same rows with every value moved one
    ulp either way (no longer an integer / a ratio), -0.0, counts past the tables (256, 128), and
    NaN, all against the wide-layout kernel and the oracle."""
    z = np.load(os.path.join(ROOT, "bench_assets", "rf100_d20.npz"))
    arr = _arrays(z)
    f = ops.Forest(arr, 15, z["mean"], z["scale"])
    g = ops.Forest(arr, 15, z["mean"], z["scale"])
    g.set_variant(0)
    rng = np.random.default_rng(8)
    base = np.vstack([z["check_X"]] * 8)
    up, dn = np.nextafter(base, np.inf), np.nextafter(base, -np.inf)
    X = np.vstack([base, up, dn])
    m = rng.random(X.shape) < 0.02
    X[m] = -0.0
    big = rng.random(len(X)) < 0.01
    X[big, 9] = 256.0 + rng.integers(0, 3, big.sum())  # past both tables
    X[big, 10] = np.round(X[big, 10] * X[big, 9]) / X[big, 9]
    X[rng.random(X.shape) < 0.002] = np.nan
    Xd = T(X, torch.float64, dev)
    p = f.predict(Xd).cpu().numpy()
    np.testing.assert_array_equal(p, g.predict(Xd).cpu().numpy())
    sel = rng.choice(len(X), 3000, replace=False)
    np.testing.assert_array_equal(p[sel], oracle.forest_predict(X[sel], arr, z["mean"], z["scale"]))
    pc = f.predict(T(z["check_X"], torch.float64, dev)).cpu().numpy()  # unperturbed: sklearn's own output
    np.testing.assert_array_equal(pc, z["check_proba"])
