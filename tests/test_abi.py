"""The C ABI surface (no GPU): libfdx.so loads, exports exactly what include/fdx.h
declares, the ctypes signatures cover every declaration, and host-only entry points work."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fdx.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fdx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("fdx_customer_windows", "fdx_terminal_windows", "fdx_rekey", "fdx_forest_predict",
                 "fdx_time_flags", "fdx_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from fdx import _lib

    L = _lib.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert set(_lib.SIGNATURES) == set(declared_functions())
    assert L.fdx_abi_version() == 2


def test_error_path_without_gpu():
    from fdx import _lib

    L = _lib.load()
    rc = L.fdx_customer_windows(None, None, None, 1, 1, None, 0, None, None, None)
    assert rc == -1
    assert b"window" in L.fdx_last_error()
    assert L.fdx_rekey_workspace_size(1000, 16) > 0


def _pack(z):
    from fdx import _lib

    L = _lib.load()
    a = {k: np.ascontiguousarray(z[k]) for k in ("node_offsets", "left", "right", "feature", "threshold",
                                                  "missing_left", "value1")}
    nt = len(a["node_offsets"]) - 1
    total = int(a["node_offsets"][-1])
    desc = _lib.ForestDesc(nt, 15, a["node_offsets"].ctypes.data, a["left"].ctypes.data,
                           a["right"].ctypes.data, a["feature"].ctypes.data, a["threshold"].ctypes.data,
                           a["missing_left"].ctypes.data, a["value1"].ctypes.data, None, None)
    nodes = np.zeros(total, np.uint64)
    orig = np.zeros(total, np.int32)
    root = np.zeros(nt, np.int32)
    rc = L.fdx_forest_pack(ctypes.byref(desc), nodes.ctypes.data, orig.ctypes.data, root.ctypes.data)
    assert rc == 0, L.fdx_last_error()
    return nodes, orig, root


def _walk_packed(nodes, orig, root, z32):
    """numpy model of the kernel's traversal over the packed nodes (float32 compares)."""
    n, nt = z32.shape[0], len(root)
    acc = np.zeros(n)
    leaves = np.zeros((n, nt), np.int32)
    hi = (nodes >> np.uint64(32)).astype(np.uint32)
    thr = (nodes & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32)
    vals = nodes.view(np.float64)
    for t in range(nt):
        p = np.full(n, root[t], np.int64)
        while True:
            h = hi[p]
            internal = (h & 0x80000000) != 0
            if not internal.any():
                break
            f = ((h >> 24) & 63).astype(np.int64)
            x = z32[np.arange(n), np.minimum(f, z32.shape[1] - 1)]
            left = np.where(np.isnan(x), (h >> 30) & 1, x <= thr[p]).astype(bool)
            rel = (h & 0xFFFFFF).astype(np.int64) // 8
            p = np.where(internal, np.where(left, p + 1, p + rel), p)
        acc = acc + vals[p]
        leaves[:, t] = orig[p]
    return acc / nt, leaves


@pytest.mark.parametrize("name", ["forest_dt2.npz", "forest_rf5d8.npz", "forest_rf3.npz"])
def test_forest_packing_reproduces_sklearn(golden, name):
    """Round-toward--inf float32 thresholds + packed pre-order layout give sklearn's exact
    leaves and probabilities (checked on the host with a numpy walk of the packed nodes)."""
    z = golden(name)
    nodes, orig, root = _pack(z)
    z32 = ((z["X"] - z["mean"]) / z["scale"]).astype(np.float32)
    proba, leaves = _walk_packed(nodes, orig, root, z32)
    np.testing.assert_array_equal(leaves, z["leaves"])
    np.testing.assert_array_equal(proba, z["proba"])


def test_threshold_round_down_edge_cases():
    """x32 <= thr64  <=>  x32 <= round_down_f32(thr64) for thresholds between floats."""
    from fdx import _lib

    thr = np.array([0.1, -0.1, 1e-40, -1e-40, 3.4e38, 1.0, 0.5 + 2**-30, -2.5 - 2**-40], np.float64)
    n = len(thr)
    z = dict(node_offsets=np.arange(0, 3 * n + 1, 3, dtype=np.int64),
             left=np.tile(np.array([1, -1, -1], np.int64), n), right=np.tile(np.array([2, -1, -1], np.int64), n),
             feature=np.zeros(3 * n, np.int64), threshold=np.repeat(thr, 3), missing_left=np.zeros(3 * n, np.uint8),
             value1=np.tile(np.array([0.0, 1.0, 0.0]), n))
    nodes, orig, root = _pack(z)
    cand = np.concatenate([np.nextafter(thr.astype(np.float32), np.float32(np.inf)), thr.astype(np.float32),
                           np.nextafter(thr.astype(np.float32), np.float32(-np.inf))])
    z32 = np.zeros((len(cand), 15), np.float32)
    z32[:, 0] = cand
    proba, leaves = _walk_packed(nodes, orig, root, z32)
    expect = np.stack([(cand.astype(np.float64) <= t) for t in thr], axis=1)  # left leaf = node 1
    np.testing.assert_array_equal(leaves == 1, expect)
    _ = _lib


def test_feature_table_layouts_match_the_header():
    """The featurized table's two layouts (include/fdx.h): the 80-byte fdx_feature_row record
    (FeatureRecords' views) and the slot-order columns at FDX_FEATURE_COL(c, cap)
    (FeatureTable's views) -- checked on CPU tensors by writing through the C layout and
    reading through the Python views."""
    import torch

    from fdx import ops

    class Row(ctypes.Structure):  # the header's struct, field for field
        _fields_ = [("cust_nb", ctypes.c_int32 * 3), ("term_nb", ctypes.c_int32 * 3),
                    ("cust_avg", ctypes.c_double * 3), ("term_risk", ctypes.c_double * 3),
                    ("weekend", ctypes.c_uint8), ("night", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 2),
                    ("row", ctypes.c_int32)]

    assert ctypes.sizeof(Row) == ops.FeatureRecords.BYTES == 80
    rec = ops.FeatureRecords(3, "cpu")
    for r in range(3):
        x = Row((ctypes.c_int32 * 3)(r, r + 1, r + 2), (ctypes.c_int32 * 3)(10 + r, 11, 12),
                (ctypes.c_double * 3)(0.5 + r, 1.5, 2.5), (ctypes.c_double * 3)(0.25, 0.125 * r, 1.0),
                r % 2, 1, (ctypes.c_uint8 * 2)(0, 0), 100 + r)
        rec.buf[r] = torch.frombuffer(bytearray(bytes(x)), dtype=torch.uint8)
    c = rec.columns()
    assert c["cust_nb"][:, 2].tolist() == [2, 3, 4] and c["term_nb"][0].tolist() == [10, 11, 12]
    assert c["cust_avg"][0].tolist() == [0.5, 1.5, 2.5] and c["term_risk"][1].tolist() == [0.0, 0.125, 0.25]
    assert c["weekend"].tolist() == [0, 1, 0] and c["night"].tolist() == [1, 1, 1]
    assert c["row"].tolist() == [100, 101, 102]

    def col(c_, cap):  # FDX_FEATURE_COL of include/fdx.h
        return c_ * 4 * cap if c_ < 6 else (24 * cap + (c_ - 6) * 8 * cap if c_ < 12 else
                                            (72 * cap if c_ == 12 else 76 * cap))

    src = open(HEADER).read()
    assert "#define FDX_FEATURE_TABLE_BYTES(cap) ((int64_t)78 * (cap))" in src
    t = ops.FeatureTable(100, "cpu")
    cap = t.cap
    assert cap % 64 == 0 and cap >= 100 and t.buf.numel() == 78 * cap
    raw = t.buf.numpy()
    for w in range(3):
        raw[col(w, cap):col(w, cap) + 4 * cap].view(np.int32)[:] = np.arange(cap) + 1000 * w
        raw[col(3 + w, cap):col(3 + w, cap) + 4 * cap].view(np.int32)[:] = -np.arange(cap) - w
        raw[col(6 + w, cap):col(6 + w, cap) + 8 * cap].view(np.float64)[:] = np.arange(cap) / 8 + w
        raw[col(9 + w, cap):col(9 + w, cap) + 8 * cap].view(np.float64)[:] = np.arange(cap) / 16 - w
    raw[col(12, cap):col(12, cap) + 4 * cap].view(np.int32)[:] = np.arange(cap) * 3
    raw[col(13, cap):col(13, cap) + 2 * cap].reshape(cap, 2)[:] = np.stack([np.arange(cap) % 2, 1 - np.arange(cap) % 2], 1)
    c = t.columns(70)
    for w in range(3):
        assert c["cust_nb"][w].tolist() == list(range(1000 * w, 1000 * w + 70))
        assert c["term_nb"][w].tolist() == [-i - w for i in range(70)]
        assert c["cust_avg"][w].tolist() == [i / 8 + w for i in range(70)]
        assert c["term_risk"][w].tolist() == [i / 16 - w for i in range(70)]
    assert c["row"].tolist() == [3 * i for i in range(70)]
    assert c["weekend"].tolist() == [i % 2 for i in range(70)] and c["night"].tolist() == [1 - i % 2 for i in range(70)]
