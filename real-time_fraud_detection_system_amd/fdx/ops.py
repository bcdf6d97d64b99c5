"""Device-tensor wrappers over the libfdx C ABI.

Every function takes / returns torch tensors resident on the GPU and enqueues work on
torch's current HIP stream (``torch.cuda.current_stream().cuda_stream`` is the
``hipStream_t`` passed to the C ABI).  PyTorch is used only for device memory and
streams; all arithmetic happens in the HIP kernels of libfdx.so.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import FdxError, check

NS_PER_DAY = 86_400 * 1_000_000_000


def require_gpu() -> torch.device:
    if not torch.cuda.is_available():
        raise FdxError("fdx requires a ROCm GPU (MI355X); no CPU fallback exists")
    _lib.load()
    return torch.device("cuda", torch.cuda.current_device())


def _s(stream=None) -> int:
    return (stream or torch.cuda.current_stream()).cuda_stream


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _dev(t: torch.Tensor, dtype, name):
    if t.device.type != "cuda":
        raise FdxError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise FdxError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise FdxError(f"{name} must be contiguous")
    return t


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def _fresh(device):
    """The default allocator of the ops below: a new tensor per call (torch's caching allocator)."""
    return lambda _name, numel, dtype: torch.empty(max(int(numel), 0), dtype=dtype, device=device)


class Arena:
    """Device buffers kept across calls of a repeated step (FraudPipeline.run_fused): alloc(name,
    numel, dtype) returns a view of the buffer `name`, reallocated only when a larger one is
    needed, so a steady stream of same-sized steps allocates nothing.  At configs[3] on one GPU
    (708M tx, ~240 GB live) the caching allocator otherwise freed and re-mapped blocks inside
    every step (2 OOM retries and 14 hipMallocs per 3 steps: 2.5 s per step instead of ~0.5,
    profiles/r06n_*).  The caller orders the reuse: a buffer is handed out again only to work
    that the stream joins place after every use of its previous contents."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._buf = {}

    _esz = {}

    def __call__(self, name: str, numel: int, dtype) -> torch.Tensor:
        esz = Arena._esz.get(dtype)
        if esz is None:
            esz = Arena._esz[dtype] = torch.empty((), dtype=dtype).element_size()
        nbytes = max(int(numel), 1) * esz
        t = self._buf.get(name)
        if t is None or t.numel() < nbytes:
            self._buf.pop(name, None)  # (freed first: the old and the new one need not coexist)
            t = self._buf[name] = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return t[:int(numel) * esz].view(dtype)

    def scope(self, prefix: str, shared=()):
        """alloc for one call site: names get `prefix.`, except those in `shared` (buffers two call
        sites may reuse because their uses are ordered, e.g. the two re-keys' scratch)."""
        return lambda name, numel, dtype: self(name if name in shared else f"{prefix}.{name}", numel, dtype)

    @property
    def nbytes(self) -> int:
        return sum(t.numel() for t in self._buf.values())


def key_bits_for(n_keys: int) -> int:
    return max(int(n_keys) - 1, 0).bit_length()


# ----------------------------------------------------------------------------- flags
def time_flags(ts_ns: torch.Tensor, mode: int = _lib.FDX_FLAGS_NOTEBOOK, stream=None):
    _dev(ts_ns, torch.int64, "ts_ns")
    n = ts_ns.numel()
    pad = (n + 7) // 8 * 8
    we = torch.empty(pad, dtype=torch.uint8, device=ts_ns.device)
    ni = torch.empty(pad, dtype=torch.uint8, device=ts_ns.device)
    check(_lib.load().fdx_time_flags(_ptr(ts_ns), n, mode, _ptr(we), _ptr(ni), _s(stream)), "fdx_time_flags")
    return we[:n], ni[:n]


# ---------------------------------------------------------------------------- re-key
def rekey(keys: torch.Tensor, n_keys: int, stream=None, want_sorted_keys: bool = False):
    """Stable grouping by key: returns (perm int32, seg_off int64[n_keys+1], sorted_keys|None)."""
    _dev(keys, torch.int32, "keys")
    n = keys.numel()
    kb = key_bits_for(n_keys)
    dev = keys.device
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    seg = torch.empty(n_keys + 1, dtype=torch.int64, device=dev)
    sk = torch.empty(n, dtype=torch.int32, device=dev) if want_sorted_keys else None
    L = _lib.load()
    ws = workspace(L.fdx_rekey_workspace_size(n, kb), dev)
    check(L.fdx_rekey(_ptr(keys), n, kb, int(n_keys), _ptr(perm), _ptr(sk), _ptr(seg), _ptr(ws),
                      ws.numel(), _s(stream)), "fdx_rekey")
    return perm, seg, sk


def rekey_payload(keys: torch.Tensor, n_keys: int, pay0: torch.Tensor | None = None, pay1: torch.Tensor | None = None,
                  flag: torch.Tensor | None = None, stream=None, seg_off: bool = True, bad: torch.Tensor | None = None,
                  alloc=None, keys_out: torch.Tensor | None = None, hist0: torch.Tensor | None = None):
    """rekey that also moves up to two 8-byte columns (int64 / float64, input row order) into
    grouped order inside the radix passes; flag (uint8 per row) is packed into bit 31 of perm.
    bad (int32 device scalar): receives the number of keys outside [0, n_keys), counted in the
    first radix pass (fdx_rekey_payload_checked; see KeyRangeCheck.from_count).
    keys_out (int32 [n], 16-byte aligned): receives the sorted keys instead of seg_off being
    derived (fdx_rekey_payload_keys; segment_offsets_sorted derives it later, so that another
    re-key sharing the scratch may start in between).  hist0: the first pass's table from
    rekey_hist0 over the same keys (fdx_rekey_payload_hist0; the id-range count was taken there,
    so bad must be None).
    -> (perm int32, seg_off int64[n_keys+1] (None with seg_off=False or keys_out), pay0 grouped |
    None, pay1 grouped | None).  alloc: see Arena (outputs "perm", "seg", "pay0", "pay1", scratch
    "rekey_ws")."""
    _dev(keys, torch.int32, "keys")
    n = keys.numel()
    dev = keys.device
    for t, nm in ((pay0, "pay0"), (pay1, "pay1")):
        if t is not None:
            if t.device.type != "cuda" or t.element_size() != 8 or not t.is_contiguous() or t.numel() != n:
                raise FdxError(f"{nm} must be a contiguous 8-byte GPU column of {n} rows")
    if pay1 is not None and pay0 is None:
        raise FdxError("pay1 needs pay0")
    if flag is not None:
        _dev(flag, torch.uint8, "flag")
    kb = max(key_bits_for(n_keys), 1)
    A = alloc or _fresh(dev)
    perm = A("perm", n, torch.int32)
    seg = A("seg", n_keys + 1, torch.int64) if seg_off and keys_out is None else None
    o0 = A("pay0", n, pay0.dtype) if pay0 is not None else None
    o1 = A("pay1", n, pay1.dtype) if pay1 is not None else None
    L = _lib.load()
    ws = A("rekey_ws", max(L.fdx_rekey_payload_workspace_size(n, kb, (pay0 is not None) + (pay1 is not None)), 1),
           torch.uint8)
    if hist0 is not None:
        if bad is not None or keys_out is not None:
            raise FdxError("hist0 takes neither bad (counted by rekey_hist0) nor keys_out")
        if hist0.numel() < L.fdx_rekey_hist0_size(n, kb):
            raise FdxError("hist0 is smaller than fdx_rekey_hist0_size")
        check(L.fdx_rekey_payload_hist0(_ptr(keys), n, kb, int(n_keys), _ptr(flag), _ptr(pay0), _ptr(pay1), _ptr(perm),
                                        _ptr(seg), _ptr(o0), _ptr(o1), _ptr(hist0), _ptr(ws), ws.numel(), _s(stream)),
              "fdx_rekey_payload_hist0")
    elif keys_out is not None:
        _dev(keys_out, torch.int32, "keys_out")
        if keys_out.numel() < n:
            raise FdxError(f"keys_out holds {keys_out.numel()} keys, {n} needed")
        if bad is not None:
            _dev(bad, torch.int32, "bad")
        check(L.fdx_rekey_payload_keys(_ptr(keys), n, kb, int(n_keys), _ptr(flag), _ptr(pay0), _ptr(pay1), _ptr(perm),
                                       _ptr(keys_out), _ptr(o0), _ptr(o1), _ptr(bad), _ptr(ws), ws.numel(), _s(stream)),
              "fdx_rekey_payload_keys")
    elif bad is not None:
        _dev(bad, torch.int32, "bad")
        check(L.fdx_rekey_payload_checked(_ptr(keys), n, kb, int(n_keys), _ptr(flag), _ptr(pay0), _ptr(pay1),
                                          _ptr(perm), _ptr(seg), _ptr(o0), _ptr(o1), _ptr(bad), _ptr(ws), ws.numel(),
                                          _s(stream)), "fdx_rekey_payload_checked")
    else:
        check(L.fdx_rekey_payload(_ptr(keys), n, kb, int(n_keys), _ptr(flag), _ptr(pay0), _ptr(pay1), _ptr(perm),
                                  _ptr(seg), _ptr(o0), _ptr(o1), _ptr(ws), ws.numel(), _s(stream)), "fdx_rekey_payload")
    return perm, seg, o0, o1


def rekey_hist0(keys: torch.Tensor, n_keys: int, stream=None, bad: torch.Tensor | None = None, alloc=None):
    """The first radix pass's scanned digit table of rekey_payload(keys, n_keys, ...), computed
    ahead of it (fdx_rekey_hist0); bad (int32 device scalar, optional): the id-range count.
    -> uint8 buffer for rekey_payload(hist0=).  alloc: see Arena (output "hist0")."""
    _dev(keys, torch.int32, "keys")
    n = keys.numel()
    kb = max(key_bits_for(n_keys), 1)
    L = _lib.load()
    A = alloc or _fresh(keys.device)
    h = A("hist0", max(L.fdx_rekey_hist0_size(n, kb), 1), torch.uint8)
    if bad is not None:
        _dev(bad, torch.int32, "bad")
    check(L.fdx_rekey_hist0(_ptr(keys), n, kb, int(n_keys), _ptr(h), h.numel(), _ptr(bad), _s(stream)),
          "fdx_rekey_hist0")
    return h


def segment_offsets_sorted(sorted_keys: torch.Tensor, n_keys: int, stream=None, alloc=None, n: int | None = None):
    """seg_off int64 [n_keys + 1] from keys sorted ascending (the first n of sorted_keys; rekey's
    seg_off), one pass (fdx_segment_offsets_sorted).  alloc: see Arena (output "seg")."""
    _dev(sorted_keys, torch.int32, "sorted_keys")
    n = sorted_keys.numel() if n is None else int(n)
    A = alloc or _fresh(sorted_keys.device)
    seg = A("seg", int(n_keys) + 1, torch.int64)
    check(_lib.load().fdx_segment_offsets_sorted(_ptr(sorted_keys), n, int(n_keys), _ptr(seg), _s(stream)),
          "fdx_segment_offsets_sorted")
    return seg


def key_map(keys: torch.Tensor, op: int, param: int, stream=None) -> torch.Tensor:
    """MOD: key % param, DIV: key / param, SUB: key - param (int32, on the GPU)."""
    _dev(keys, torch.int32, "keys")
    out = torch.empty_like(keys)
    check(_lib.load().fdx_key_map(_ptr(keys), keys.numel(), int(op), int(param), _ptr(out), _s(stream)),
          "fdx_key_map")
    return out


def count_out_of_range(keys: torch.Tensor, lo: int, hi: int, stream=None) -> torch.Tensor:
    """-> int32 device scalar: #keys outside [lo, hi) (asynchronous; read it after a sync)."""
    _dev(keys, torch.int32, "keys")
    out = torch.empty(1, dtype=torch.int32, device=keys.device)
    check(_lib.load().fdx_count_out_of_range(_ptr(keys), keys.numel(), int(lo), int(hi), _ptr(out), _s(stream)),
          "fdx_count_out_of_range")
    return out


class KeyRangeCheck:
    """Enqueue a key-range count now, read it after the caller's next host synchronisation
    (no extra stall): the count is copied into pinned host memory on the same stream."""

    def __init__(self, keys: torch.Tensor | None, n_keys: int, what: str = "keys", stream=None,
                 count: torch.Tensor | None = None):
        self.what, self.n_keys = what, int(n_keys)
        st = stream or torch.cuda.current_stream()
        self._host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        # count, copy and event all on `st` (the copy must follow the count kernel, and the
        # event must follow the copy), whatever torch's current stream is
        with torch.cuda.stream(st):
            self._host.copy_(count if count is not None else count_out_of_range(keys, 0, n_keys, st),
                             non_blocking=True)
            self._ev = torch.cuda.Event()
            self._ev.record(st)

    @classmethod
    def from_count(cls, count: torch.Tensor, n_keys: int, what: str = "keys", stream=None) -> "KeyRangeCheck":
        """Read a count some kernel already made on `stream` (rekey_payload(bad=...)): only the
        pinned copy is enqueued."""
        return cls(None, n_keys, what, stream, count=count)

    def check(self) -> None:
        self._ev.synchronize()
        bad = int(self._host.item())
        if bad:
            raise FdxError(f"{bad} {self.what} outside [0, {self.n_keys}): the grouping would be wrong")


def argsort_i64(keys: torch.Tensor, stream=None) -> torch.Tensor:
    _dev(keys, torch.int64, "keys")
    n = keys.numel()
    perm = torch.empty(n, dtype=torch.int32, device=keys.device)
    L = _lib.load()
    ws = workspace(L.fdx_argsort_i64_workspace_size(n), keys.device)
    check(L.fdx_argsort_i64(_ptr(keys), n, _ptr(perm), _ptr(ws), ws.numel(), _s(stream)), "fdx_argsort_i64")
    return perm


def dense_ids_i64(keys: torch.Tensor, stream=None):
    """(ids int32 [n], n_unique int64 device tensor [1]): order-preserving dense ids of int64
    keys (fdx_dense_ids_i64)."""
    _dev(keys, torch.int64, "keys")
    n = keys.numel()
    ids = torch.empty(n, dtype=torch.int32, device=keys.device)
    nu = torch.empty(1, dtype=torch.int64, device=keys.device)
    L = _lib.load()
    ws = workspace(L.fdx_dense_ids_i64_workspace_size(n), keys.device)
    check(L.fdx_dense_ids_i64(_ptr(keys), n, _ptr(ids), _ptr(nu), _ptr(ws), ws.numel(), _s(stream)),
          "fdx_dense_ids_i64")
    return ids, nu


def is_sorted_i64(keys: torch.Tensor, stream=None) -> bool:
    """Host-synchronising check (reads one int back)."""
    _dev(keys, torch.int64, "keys")
    flag = torch.empty(1, dtype=torch.int32, device=keys.device)
    check(_lib.load().fdx_is_sorted_i64(_ptr(keys), keys.numel(), _ptr(flag), _s(stream)), "fdx_is_sorted_i64")
    return bool(flag.item())


def gather(src: torch.Tensor, perm: torch.Tensor, stream=None) -> torch.Tensor:
    _dev(perm, torch.int32, "perm")
    if not src.is_contiguous():
        raise FdxError("src must be contiguous")
    out = torch.empty(perm.numel(), dtype=src.dtype, device=src.device)
    check(_lib.load().fdx_gather(_ptr(src), src.element_size(), _ptr(perm), perm.numel(), _ptr(out),
                                 _s(stream)), "fdx_gather")
    return out


def scatter(src: torch.Tensor, perm: torch.Tensor, out: torch.Tensor | None = None, stream=None):
    _dev(perm, torch.int32, "perm")
    if out is None:
        out = torch.empty(perm.numel(), dtype=src.dtype, device=src.device)
    check(_lib.load().fdx_scatter(_ptr(src), src.element_size(), _ptr(perm), perm.numel(), _ptr(out),
                                  _s(stream)), "fdx_scatter")
    return out


# --------------------------------------------------------------------------- windows
_WIN_NS = {}


def _win_ns(days: Sequence[int]):
    key = tuple(days)
    w = _WIN_NS.get(key)
    if w is None:  # (built once per window set: the step's host path calls this several times)
        days = [int(d) for d in days]
        if not 1 <= len(days) <= _lib.MAX_WINDOWS:
            raise FdxError(f"1..{_lib.MAX_WINDOWS} windows supported")
        w = _WIN_NS[key] = (ctypes.c_int64 * len(days))(*[d * NS_PER_DAY for d in days])
    return w


def customer_windows(ts_ns, amount, seg_off, windows_days=(1, 7, 30), stream=None):
    """Grouped rows -> (nb int32 [W, n], avg float64 [W, n])."""
    _dev(ts_ns, torch.int64, "ts_ns"); _dev(amount, torch.float64, "amount"); _dev(seg_off, torch.int64, "seg_off")
    n = ts_ns.numel()
    W = len(windows_days)
    nb = torch.empty((W, n), dtype=torch.int32, device=ts_ns.device)
    avg = torch.empty((W, n), dtype=torch.float64, device=ts_ns.device)
    check(_lib.load().fdx_customer_windows(_ptr(ts_ns), _ptr(amount), _ptr(seg_off), seg_off.numel() - 1, n,
                                           _win_ns(windows_days), W, _ptr(nb), _ptr(avg), _s(stream)),
          "fdx_customer_windows")
    return nb, avg


def terminal_windows(ts_ns, fraud, seg_off, delay_days=7, windows_days=(1, 7, 30), stream=None):
    """Grouped rows -> (nb int32 [W, n], risk float64 [W, n]); the kernel's scratch is a caller
    workspace (fdx_terminal_windows_workspace_size)."""
    _dev(ts_ns, torch.int64, "ts_ns"); _dev(fraud, torch.uint8, "fraud"); _dev(seg_off, torch.int64, "seg_off")
    n = ts_ns.numel()
    W = len(windows_days)
    nb = torch.empty((W, n), dtype=torch.int32, device=ts_ns.device)
    risk = torch.empty((W, n), dtype=torch.float64, device=ts_ns.device)
    L = _lib.load()
    ws = workspace(L.fdx_terminal_windows_workspace_size(n), ts_ns.device)
    check(L.fdx_terminal_windows(_ptr(ts_ns), _ptr(fraud), _ptr(seg_off), seg_off.numel() - 1, n,
                                 int(delay_days) * NS_PER_DAY, _win_ns(windows_days), W, _ptr(nb), _ptr(risk),
                                 _ptr(ws), ws.numel(), _s(stream)), "fdx_terminal_windows")
    return nb, risk


def customer_windows_scan(gts, gamount, seg_off, windows_days=(1, 7, 30), lay=None, val_is_sum: bool = False,
                          stream=None):
    """Customer windows in SCAN mode (fdx_customer_windows_scan): grouped ts / amount
    (rekey_payload outputs) -> (nb int32 [W, m], val float64 [W, m]), by grouped position
    (m = n; val = the average SUM / NB, or SUM when val_is_sum) or, with lay (an interleaved
    layout of the same segments), by slot (m = n_slots; val = SUM, what customer_windows_walk
    returns).  NB exact; the sums agree with pandas' roll_sum to ~1e-13 relative, not bit for
    bit."""
    _dev(gts, torch.int64, "gts"); _dev(gamount, torch.float64, "gamount"); _dev(seg_off, torch.int64, "seg_off")
    n = gts.numel()
    n_seg = seg_off.numel() - 1
    W = len(windows_days)
    dev = gts.device
    m = lay.n_slots if lay is not None else n
    nb = torch.empty((W, m), dtype=torch.int32, device=dev)
    val = torch.empty((W, m), dtype=torch.float64, device=dev)
    if n == 0 or m == 0:
        return nb, val
    L = _lib.load()
    ws = workspace(L.fdx_customer_windows_scan_workspace_size(n, n_seg), dev)
    if lay is not None and lay.starts is not None:  # the layout's starts: two coalesced passes
        if tuple(lay.windows_days) != tuple(int(w) for w in windows_days):
            raise FdxError("layout starts were built for other windows")
        check(L.fdx_customer_windows_scan_slots(_ptr(gamount), _ptr(seg_off), n_seg, n, _ptr(lay.sorder),
                                                _ptr(lay.goff), m, W, _ptr(lay.starts), _ptr(nb), _ptr(val),
                                                _ptr(ws), ws.numel(), _s(stream)),
              "fdx_customer_windows_scan_slots")
        return nb, val
    check(L.fdx_customer_windows_scan(_ptr(gts), _ptr(gamount), _ptr(seg_off), n_seg, n, _win_ns(windows_days), W,
                                      _ptr(lay.sorder) if lay is not None else None,
                                      _ptr(lay.goff) if lay is not None else None, m, _ptr(nb), _ptr(val),
                                      int(bool(val_is_sum or lay is not None)), _ptr(ws), ws.numel(), _s(stream)),
          "fdx_customer_windows_scan")
    return nb, val


class CustomerLayout:
    """The interleaved (lane-major) customer layout of the scoring pipeline (fdx.h).
    starts: the window starts [W * max_slots] int32 when built by customer_layout(windows_days=...)."""

    def __init__(self, sorder, goff, its, iamt, irow, n_slots, starts=None, windows_days=None):
        self.sorder, self.goff, self.its, self.iamt, self.irow, self.n_slots = sorder, goff, its, iamt, irow, n_slots
        self.starts, self.windows_days = starts, windows_days


def customer_layout(seg_off, cperm, ts_ns, amount, n_windows: int, stream=None, _slots_hint=None,
                    windows_days=None, grouped: bool = False) -> CustomerLayout:
    """windows_days: also compute the window starts in the layout kernel (for
    customer_windows_walk).  grouped: ts_ns / amount are in grouped order (rekey_payload
    outputs) and are read as sequential streams."""
    _dev(seg_off, torch.int64, "seg_off"); _dev(cperm, torch.int32, "cperm")
    _dev(ts_ns, torch.int64, "ts_ns"); _dev(amount, torch.float64, "amount")
    n_seg = seg_off.numel() - 1
    n = ts_ns.numel()
    S = 64 // int(n_windows)
    dev = ts_ns.device
    L = _lib.load()
    if n == 0:  # no rows: an empty layout (every consumer then has zero slots to process)
        z32 = torch.zeros(0, dtype=torch.int32, device=dev)
        return CustomerLayout(z32, torch.zeros(1, dtype=torch.int32, device=dev),
                              torch.zeros(0, dtype=torch.int64, device=dev),
                              torch.zeros(0, dtype=torch.float64, device=dev), z32, 0,
                              None if windows_days is None else z32,
                              None if windows_days is None else tuple(windows_days))
    max_slots = int(_slots_hint or (n + S * 4096))
    sorder = torch.empty(max(n_seg, 1), dtype=torch.int32, device=dev)
    goff = torch.empty(-(-n_seg // S) + 1, dtype=torch.int32, device=dev)
    ws = workspace(L.fdx_customer_layout_workspace_size(n_seg), dev)
    while True:
        its = torch.empty(max_slots, dtype=torch.int64, device=dev)
        iamt = torch.empty(max_slots, dtype=torch.float64, device=dev)
        irow = torch.empty(max_slots, dtype=torch.int32, device=dev)
        ns = ctypes.c_int64(0)
        if windows_days is None:
            starts = None
            fn = L.fdx_customer_layout_grouped if grouped else L.fdx_customer_layout
            rc = fn(_ptr(seg_off), n_seg, _ptr(cperm), _ptr(ts_ns), _ptr(amount), int(n_windows),
                    _ptr(sorder), _ptr(goff), _ptr(its), _ptr(iamt), _ptr(irow), max_slots,
                    ctypes.byref(ns), _ptr(ws), ws.numel(), _s(stream))
        else:
            if len(windows_days) != int(n_windows):
                raise FdxError("windows_days must have n_windows entries")
            starts = torch.empty(int(n_windows) * max_slots, dtype=torch.int32, device=dev)
            fn = L.fdx_customer_layout_starts_grouped if grouped else L.fdx_customer_layout_starts
            rc = fn(_ptr(seg_off), n_seg, _ptr(cperm), _ptr(ts_ns), _ptr(amount),
                                              _win_ns(windows_days), int(n_windows), _ptr(sorder), _ptr(goff),
                                              _ptr(its), _ptr(iamt), _ptr(irow), _ptr(starts), max_slots,
                                              ctypes.byref(ns), _ptr(ws), ws.numel(), _s(stream))
        if rc == -4 and ns.value > max_slots:
            if ns.value > S * n:  # every group pads to its longest segment: <= S slots per row
                raise FdxError(f"customer layout: {ns.value} slots for {n} rows -- inconsistent segment "
                               "offsets (keys outside [0, n_keys)?)")
            max_slots = ns.value
            continue
        check(rc, "fdx_customer_layout")
        return CustomerLayout(sorder, goff, its, iamt, irow, ns.value, starts,
                              None if windows_days is None else tuple(windows_days))


def key_segments(keys, n_keys: int, stream=None, bad: torch.Tensor | None = None, alloc=None) -> torch.Tensor:
    """seg_off int64 [n_keys + 1] of the stable grouping by key (rekey's seg_off for keys in
    [0, n_keys)) from a key histogram, no sort; bad (int32 [1], optional): out-of-range count.
    alloc: see Arena (output "seg", scratch "ksws")."""
    _dev(keys, torch.int32, "keys")
    L = _lib.load()
    dev = keys.device
    A = alloc or _fresh(dev)
    seg = A("seg", int(n_keys) + 1, torch.int64)
    ws = A("ksws", max(L.fdx_key_segments_workspace_size(int(n_keys)), 1), torch.uint8)
    check(L.fdx_key_segments(_ptr(keys), keys.numel(), int(n_keys), _ptr(seg), _ptr(bad) if bad is not None else None,
                             _ptr(ws), ws.numel(), _s(stream)), "fdx_key_segments")
    return seg


class LayoutPlan:
    """fdx_customer_layout_plan's outputs: segment order, group slot offsets, slot count."""

    def __init__(self, sorder, goff, n_slots, n_windows):
        self.sorder, self.goff, self.n_slots, self.n_windows = sorder, goff, n_slots, n_windows


def customer_layout_plan(seg_off, n_windows: int, stream=None) -> LayoutPlan:
    """The first half of customer_layout, from the segment offsets alone (host-synchronising:
    the slot count is read back)."""
    _dev(seg_off, torch.int64, "seg_off")
    n_seg = seg_off.numel() - 1
    S = 64 // int(n_windows)
    dev = seg_off.device
    L = _lib.load()
    sorder = torch.empty(max(n_seg, 1), dtype=torch.int32, device=dev)
    goff = torch.empty(-(-n_seg // S) + 1, dtype=torch.int32, device=dev)
    ws = workspace(L.fdx_customer_layout_workspace_size(n_seg), dev)
    ns = ctypes.c_int64(0)
    check(L.fdx_customer_layout_plan(_ptr(seg_off), n_seg, int(n_windows), _ptr(sorder), _ptr(goff), ctypes.byref(ns),
                                     _ptr(ws), ws.numel(), _s(stream)), "fdx_customer_layout_plan")
    return LayoutPlan(sorder, goff, ns.value, int(n_windows))


class PendingPlan:
    """customer_layout_plan_async's handle: result() waits for the stream to pass the plan
    (no earlier) and returns the LayoutPlan (re-planning synchronously if the one-launch plan
    declined)."""

    # wall time to poll the pinned result before the blocking wait: the plan lands ~1-2 ms after
    # it is enqueued at config 2 (behind the customer re-key), so the poll usually ends first
    SPIN_S = 5e-3

    def __init__(self, seg_off, n_windows, stream, alloc=None):
        self.seg_off, self.n_windows, self.stream = seg_off, int(n_windows), stream
        n_seg = seg_off.numel() - 1
        S = 64 // self.n_windows
        dev = seg_off.device
        L = _lib.load()
        A = alloc or _fresh(dev)
        self.sorder = A("sorder", max(n_seg, 1), torch.int32)
        self.goff = A("goff", -(-n_seg // S) + 1, torch.int32)
        self.ws = A("plan_ws", max(L.fdx_customer_layout_workspace_size(n_seg), 1), torch.uint8)
        # [slot count, status], -1 until the stream's copy lands (result() polls for it)
        self.host = torch.full((2,), -1, dtype=torch.int32, pin_memory=True)
        self._hv = self.host.numpy()
        st = stream or torch.cuda.current_stream()
        rc = L.fdx_customer_layout_plan_async(_ptr(seg_off), n_seg, self.n_windows, _ptr(self.sorder), _ptr(self.goff),
                                              self.host.data_ptr(), _ptr(self.ws), self.ws.numel(), _s(st))
        self.ok = rc == _lib.FDX_OK
        if not self.ok and rc != _lib.FDX_E_UNSUPPORTED:
            check(rc, "fdx_customer_layout_plan_async")
        self.ev = torch.cuda.Event()
        self.ev.record(st)

    def result(self, spin_s: float | None = None) -> LayoutPlan:
        if self.ok:
            # poll the pinned words for a bounded while before the blocking wait: the step's
            # critical stream idles until the host has read the slot count and launched the
            # layout fill, and waking from hipEventSynchronize took ~70 us (profiles/r03ad)
            # (bounded by wall time, not a poll count: a Python poll costs 0.1-0.2 us and holds the GIL)
            hv = self._hv
            t_end = time.perf_counter() + (self.SPIN_S if spin_s is None else spin_s)
            while hv[0] == -1 or hv[1] == -1:
                if time.perf_counter() > t_end:
                    self.ev.synchronize()
                    break
            if int(hv[1]) == 0:
                return LayoutPlan(self.sorder, self.goff, int(hv[0]) & 0xFFFFFFFF, self.n_windows)
        return customer_layout_plan(self.seg_off, self.n_windows, self.stream)


def customer_layout_plan_async(seg_off, n_windows: int, stream=None, alloc=None) -> PendingPlan:
    """Enqueue the layout plan without waiting for it (see PendingPlan; alloc: see Arena)."""
    _dev(seg_off, torch.int64, "seg_off")
    return PendingPlan(seg_off, n_windows, stream, alloc)


def customer_layout_fill(plan: LayoutPlan, seg_off, cperm, gts, gamt, windows_days, stream=None,
                         alloc=None) -> CustomerLayout:
    """The second half: slots and window starts of a plan from GROUPED ts / amount (alloc: see Arena)."""
    _dev(seg_off, torch.int64, "seg_off"); _dev(cperm, torch.int32, "cperm")
    _dev(gts, torch.int64, "ts_ns"); _dev(gamt, torch.float64, "amount")
    W = plan.n_windows
    if len(windows_days) != W:
        raise FdxError("windows_days must have n_windows entries")
    dev, m = gts.device, plan.n_slots
    if m > (64 // W) * max(gts.numel(), 1):  # every group pads to its longest segment: <= S slots per row
        raise FdxError(f"customer layout: {m} slots for {gts.numel()} rows -- inconsistent segment offsets "
                       "(keys outside [0, n_keys)?)")
    A = alloc or _fresh(dev)
    its = A("its", m, torch.int64)
    iamt = A("iamt", m, torch.float64)
    irow = A("irow", m, torch.int32)
    starts = A("starts", W * m, torch.int32)
    if m:
        check(_lib.load().fdx_customer_layout_fill_starts_grouped(
            _ptr(seg_off), seg_off.numel() - 1, _ptr(cperm), _ptr(gts), _ptr(gamt), _win_ns(windows_days), W,
            _ptr(plan.sorder), _ptr(plan.goff), m, _ptr(its), _ptr(iamt), _ptr(irow), _ptr(starts), _s(stream)),
            "fdx_customer_layout_fill_starts_grouped")
    return CustomerLayout(plan.sorder, plan.goff, its, iamt, irow, m, starts, tuple(windows_days))


def customer_windows_walk(lay: CustomerLayout, seg_off, stream=None, alloc=None):
    """The windows of a layout built with windows_days: (nb int32 [W, n_slots], rolling SUM
    float64 [W, n_slots]) indexed by slot (alloc: see Arena)."""
    if lay.starts is None:
        raise FdxError("layout was built without window starts")
    W = len(lay.windows_days)
    dev = lay.its.device
    A = alloc or _fresh(dev)
    nb = A("nb", W * lay.n_slots, torch.int32).view(W, lay.n_slots)
    sm = A("sum", W * lay.n_slots, torch.float64).view(W, lay.n_slots)
    if lay.n_slots == 0:
        return nb, sm
    check(_lib.load().fdx_customer_windows_walk(_ptr(lay.iamt), _ptr(seg_off), _ptr(lay.sorder), _ptr(lay.goff),
                                                seg_off.numel() - 1, lay.n_slots, W, _ptr(lay.starts), _ptr(nb),
                                                _ptr(sm), _s(stream)),
          "fdx_customer_windows_walk")
    return nb, sm


def customer_windows_interleaved(lay: CustomerLayout, seg_off, windows_days=(1, 7, 30), stream=None):
    """-> (nb int32 [W, n_slots], rolling SUM float64 [W, n_slots]) indexed by slot;
    the average is sum / nb (done by forest_prepare_grouped(val_is_sum=True))."""
    W = len(windows_days)
    dev = lay.its.device
    nb = torch.empty((W, lay.n_slots), dtype=torch.int32, device=dev)
    avg = torch.empty((W, lay.n_slots), dtype=torch.float64, device=dev)
    check(_lib.load().fdx_customer_windows_interleaved(_ptr(lay.its), _ptr(lay.iamt), _ptr(seg_off), _ptr(lay.sorder),
                                                       _ptr(lay.goff), seg_off.numel() - 1, lay.n_slots,
                                                       _win_ns(windows_days), W, _ptr(nb), _ptr(avg), _s(stream)),
          "fdx_customer_windows_interleaved")
    return nb, avg


def terminal_windows_compact(gts, seg_off, rows=None, gfraud=None, delay_days=7, windows_days=(1, 7, 30),
                             runs: bool = False, stream=None, alloc=None):
    """terminal_windows_grouped's count records by row in the COMPACT format (3 windows): an
    int64 [5 n] array, row r's 16-byte record at words [2 r, 2 r + 2), the overflow area
    [2 n, 5 n) (fdx.h fdx_terminal_windows_grouped_compact).  compact_records_unpack turns it
    into the [n, 3] records (alloc: see Arena)."""
    _dev(gts, torch.int64, "gts"); _dev(seg_off, torch.int64, "seg_off")
    if rows is not None:
        _dev(rows, torch.int32, "rows")
    if gfraud is not None:
        _dev(gfraud, torch.uint8, "gfraud")
    if rows is None and gfraud is None:
        raise FdxError("fraud comes from gfraud or from bit 31 of rows")
    if len(windows_days) != 3:
        raise FdxError("compact records hold 3 windows")
    n = gts.numel()
    A = alloc or _fresh(gts.device)
    rec = A("rec", max(5 * n, 2), torch.int64)  # 256-byte aligned
    scratch = A("scratch", max(n, 1), torch.int32)
    check(_lib.load().fdx_terminal_windows_grouped_compact(_ptr(gts), _ptr(gfraud), _ptr(rows), _ptr(seg_off),
                                                           seg_off.numel() - 1, n, int(delay_days) * NS_PER_DAY,
                                                           _win_ns(windows_days), 3, int(bool(runs)), _ptr(rec),
                                                           _ptr(scratch), _s(stream)),
          "fdx_terminal_windows_grouped_compact")
    return rec


def terminal_windows_grouped(gts, seg_off, rows=None, gfraud=None, delay_days=7, windows_days=(1, 7, 30),
                             runs: bool = False, records: bool = True, stream=None):
    """Terminal windows over grouped inputs (rekey_payload(terminal, ts, flag=fraud) outputs):
    gts = grouped ts; fraud from gfraud (grouped uint8) or bit 31 of rows; record of grouped
    position q written at row rows[q] & 0x7FFFFFFF (rows None: at q).  records: count records
    int64 [n, W]; else (nb int32 [W, n], risk float64 [W, n]) at grouped positions."""
    _dev(gts, torch.int64, "gts"); _dev(seg_off, torch.int64, "seg_off")
    if rows is not None:
        _dev(rows, torch.int32, "rows")
    if gfraud is not None:
        _dev(gfraud, torch.uint8, "gfraud")
    if rows is None and gfraud is None:
        raise FdxError("fraud comes from gfraud or from bit 31 of rows")
    n = gts.numel()
    W = len(windows_days)
    dev = gts.device
    scratch = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    L = _lib.load()
    args = (_ptr(gts), _ptr(gfraud), _ptr(rows), _ptr(seg_off), seg_off.numel() - 1, n, int(delay_days) * NS_PER_DAY,
            _win_ns(windows_days), W, int(bool(runs)))
    if records:
        rec = torch.empty((n, W), dtype=torch.int64, device=dev)
        check(L.fdx_terminal_windows_grouped(*args, None, None, _ptr(rec), _ptr(scratch), _s(stream)),
              "fdx_terminal_windows_grouped")
        return rec
    nb = torch.empty((W, n), dtype=torch.int32, device=dev)
    risk = torch.empty((W, n), dtype=torch.float64, device=dev)
    check(L.fdx_terminal_windows_grouped(*args, _ptr(nb), _ptr(risk), None, _ptr(scratch), _s(stream)),
          "fdx_terminal_windows_grouped")
    return nb, risk


def invert_perm(perm: torch.Tensor, stream=None) -> torch.Tensor:
    _dev(perm, torch.int32, "perm")
    inv = torch.empty_like(perm)
    check(_lib.load().fdx_invert_perm(_ptr(perm), perm.numel(), _ptr(inv), _s(stream)), "fdx_invert_perm")
    return inv


# ----------------------------------------------------------------------------- scale
def standard_scale(X: torch.Tensor, mean: torch.Tensor | None, scale: torch.Tensor | None, stream=None):
    """(X - mean) / scale in float64; X is a 2-D float64 GPU tensor (any strides)."""
    if X.dtype != torch.float64 or X.dim() != 2 or X.device.type != "cuda":
        raise FdxError("X must be a 2-D float64 GPU tensor")
    n, nf = X.shape
    out = torch.empty((n, nf), dtype=torch.float64, device=X.device)
    check(_lib.load().fdx_standard_scale(_ptr(X), n, nf, X.stride(0), X.stride(1), _ptr(mean), _ptr(scale),
                                         _ptr(out), out.stride(0), out.stride(1), _s(stream)),
          "fdx_standard_scale")
    return out


# ---------------------------------------------------------------------------- forest
class Forest:
    """A tree ensemble uploaded to the GPU (immutable; share it across streams)."""

    def __init__(self, arrays: dict, n_features: int, mean=None, scale=None, stream=None):
        require_gpu()
        a = {
            "node_offsets": np.ascontiguousarray(arrays["node_offsets"], np.int64),
            "children_left": np.ascontiguousarray(arrays["left"], np.int64),
            "children_right": np.ascontiguousarray(arrays["right"], np.int64),
            "feature": np.ascontiguousarray(arrays["feature"], np.int64),
            "threshold": np.ascontiguousarray(arrays["threshold"], np.float64),
            "missing_go_to_left": np.ascontiguousarray(arrays["missing_left"], np.uint8),
            "value1": np.ascontiguousarray(arrays["value1"], np.float64),
        }
        self._keep = a
        self.n_trees = len(a["node_offsets"]) - 1
        self.n_features = int(n_features)
        m = None if mean is None else np.ascontiguousarray(mean, np.float64)
        s = None if scale is None else np.ascontiguousarray(scale, np.float64)
        self._keep_scaler = (m, s)
        pp = lambda x: None if x is None else x.ctypes.data
        desc = _lib.ForestDesc(self.n_trees, self.n_features, pp(a["node_offsets"]), pp(a["children_left"]),
                               pp(a["children_right"]), pp(a["feature"]), pp(a["threshold"]),
                               pp(a["missing_go_to_left"]), pp(a["value1"]), pp(m), pp(s))
        h = ctypes.c_void_p()
        L = _lib.load()
        check(L.fdx_forest_create(ctypes.byref(desc), ctypes.byref(h), _s(stream)), "fdx_forest_create")
        self._h = h
        nt, nf, nn, nc = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
        check(L.fdx_forest_info(h, ctypes.byref(nt), ctypes.byref(nf), ctypes.byref(nn), ctypes.byref(nc)))
        self.n_nodes, self.n_chunks = nn.value, nc.value
        v = ctypes.c_int32()
        check(L.fdx_forest_get_variant(h, ctypes.byref(v)), "fdx_forest_get_variant")
        self.variant = v.value  # the library default (rank layout when the forest fits it)
        # bumped by every call that may re-lay the device buffers (a refused set_variant re-installs
        # the previous layout too): a captured HIP graph (StreamScorer.score_graph) holds their
        # addresses and is captured again when the epoch moved
        self.epoch = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.fdx_forest_destroy(h)
            self._h = None

    def set_variant(self, variant: int) -> None:
        self.epoch += 1
        L = _lib.load()
        check(L.fdx_forest_set_variant(self._h, int(variant)), "fdx_forest_set_variant")
        nt, nf, nn, nc = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
        check(L.fdx_forest_info(self._h, ctypes.byref(nt), ctypes.byref(nf), ctypes.byref(nn), ctypes.byref(nc)))
        self.n_chunks = nc.value
        self.variant = int(variant)

    def set_range_rows(self, rows: int) -> None:
        """rows per traversal range (fdx_forest_set_range_rows; 0 = the default)"""
        self.epoch += 1
        check(_lib.load().fdx_forest_set_range_rows(self._h, int(rows)), "fdx_forest_set_range_rows")

    def traverse_launches(self, n: int, want_leaves: bool = False) -> int:
        """tree-walk kernel launches of one traversal of n rows (fdx_forest_traverse_launches)"""
        k = ctypes.c_int32()
        check(_lib.load().fdx_forest_traverse_launches(self._h, int(n), int(bool(want_leaves)), ctypes.byref(k)),
              "fdx_forest_traverse_launches")
        return k.value

    def workspace_size(self, n: int) -> int:
        return int(_lib.load().fdx_forest_workspace_size(self._h, int(n)))

    def workspace_size_max(self, n: int) -> int:
        """one workspace for every batch of up to n rows (small batches' fast path included)"""
        return int(_lib.load().fdx_forest_workspace_size_max(self._h, int(n)))

    def predict(self, X: torch.Tensor, want_leaves: bool = False, ws: torch.Tensor | None = None,
                out: torch.Tensor | None = None, stream=None):
        """X: float64 GPU tensor [n, n_features] (any strides).  Returns proba (and leaves)."""
        if X.dtype != torch.float64 or X.dim() != 2 or X.device.type != "cuda":
            raise FdxError("X must be a 2-D float64 GPU tensor")
        n, nf = X.shape
        if nf != self.n_features:
            raise FdxError(f"X has {nf} features, forest expects {self.n_features}")
        proba = out if out is not None else torch.empty(n, dtype=torch.float64, device=X.device)
        leaves = torch.empty((n, self.n_trees), dtype=torch.int32, device=X.device) if want_leaves else None
        need = self.workspace_size(n)
        if ws is None:
            ws = workspace(need, X.device)
        check(_lib.load().fdx_forest_predict(self._h, _ptr(X), n, X.stride(0), X.stride(1), _ptr(proba),
                                             _ptr(leaves), _ptr(ws), ws.numel(), _s(stream)),
              "fdx_forest_predict")
        return (proba, leaves) if want_leaves else proba


def forest_prepare(forest: "Forest", X: torch.Tensor, ws: torch.Tensor, stream=None):
    n = X.shape[0]
    check(_lib.load().fdx_forest_prepare(forest._h, _ptr(X), n, X.stride(0), X.stride(1), _ptr(ws), ws.numel(),
                                         _s(stream)), "fdx_forest_prepare")


def forest_prepare_features(forest: "Forest", f, amount: torch.Tensor, ws: torch.Tensor, W: int,
                            with_terminal: bool = True, stream=None):
    """Fused assemble + scale into the forest workspace (float32 rows) from a
    pipeline.Features; with_terminal=False leaves the terminal columns for the reply path."""
    n = amount.numel()
    t = with_terminal
    check(_lib.load().fdx_forest_prepare_features(
        forest._h, n, W, _ptr(amount), _ptr(f.weekend), _ptr(f.night), _ptr(f.cust_perm), _ptr(f.cust_nb),
        _ptr(f.cust_avg), _ptr(f.term_perm) if t else None, _ptr(f.term_nb) if t else None,
        _ptr(f.term_risk) if t else None, _ptr(ws), ws.numel(), _s(stream)), "fdx_forest_prepare_features")


def forest_prepare_reply(forest: "Forest", reply: torch.Tensor, perm: torch.Tensor, W: int, col0: int,
                         ws: torch.Tensor, stream=None):
    check(_lib.load().fdx_forest_prepare_reply(forest._h, _ptr(reply), _ptr(perm), perm.numel(), W, col0,
                                               _ptr(ws), ws.numel(), _s(stream)), "fdx_forest_prepare_reply")


def forest_clear_flag(forest: "Forest", n: int, ws: torch.Tensor, stream=None) -> None:
    """clear the NaN flag of a workspace for n rows (for forest_prepare_grouped(flag_cleared=True))"""
    check(_lib.load().fdx_forest_clear_flag(forest._h, int(n), _ptr(ws), ws.numel(), _s(stream)),
          "fdx_forest_clear_flag")


def forest_prepare_grouped(forest: "Forest", flags_mode: int, cts, camt, cnb, cavg, cperm, term_inv, term_rec,
                           ws: torch.Tensor, stream=None, n=None, val_is_sum: bool = False, term_compact: bool = False,
                           rows_out=None, flag_cleared: bool = False):
    """cavg holds averages, or rolling sums when val_is_sum (interleaved customer path);
    term_compact: term_rec is terminal_windows_compact's array; rows_out: the featurized table
    written by the same pass -- a FeatureRecords (by input row) or a FeatureTable (columns by
    scoring slot, capacity >= n); flag_cleared: forest_clear_flag ran on this workspace before
    (stream-ordered before this call), so the call does not clear it itself."""
    n = cts.numel() if n is None else int(n)
    W = cnb.shape[0]
    opts = (1 if val_is_sum else 0) | (4 if term_compact else 0) | (8 if flag_cleared else 0)
    out, cap, order = None, 0, 0
    if rows_out is not None:
        if not isinstance(rows_out, (FeatureRecords, FeatureTable)):
            raise TypeError("rows_out must be a FeatureRecords or a FeatureTable")
        if isinstance(rows_out, FeatureTable) and rows_out.cap < n:
            raise ValueError(f"the feature table holds {rows_out.cap} slots < {n}")
        out, cap, order = rows_out.buf, rows_out.cap, rows_out.order
    check(_lib.load().fdx_forest_prepare_grouped_rows(forest._h, n, W, int(flags_mode), opts, _ptr(cts),
                                                      _ptr(camt), _ptr(cnb),
                                                      _ptr(cavg), _ptr(cperm), _ptr(term_inv), _ptr(term_rec),
                                                      _ptr(out), cap, order, _ptr(ws), ws.numel(), _s(stream)),
          "fdx_forest_prepare_grouped_rows")


class FeatureRecords:
    """The featurized table by INPUT row: fdx_feature_row records (include/fdx.h), 80 bytes each
    -- the 14 feature columns of the reference's table in SURVEY.md §8(d)'s compact form plus
    the row index; record r = transaction r (time order).  columns(): views, no copy."""
    order = _lib.FDX_ROWS_INPUT_ORDER
    BYTES = 80

    def __init__(self, n_rows: int, device):
        self.cap = int(n_rows)
        self.buf = torch.empty((self.cap, self.BYTES), dtype=torch.uint8, device=device)

    def columns(self) -> dict:
        i32, f64 = self.buf.view(torch.int32), self.buf.view(torch.float64)
        return {"cust_nb": i32[:, 0:3].T, "term_nb": i32[:, 3:6].T, "cust_avg": f64[:, 3:6].T,
                "term_risk": f64[:, 6:9].T, "weekend": self.buf[:, 72], "night": self.buf[:, 73], "row": i32[:, 19]}


class FeatureTable:
    """The featurized table by SCORING SLOT, as columns (FDX_FEATURE_COL layout of include/fdx.h,
    one buffer): each column written coalesced by the assembly pass; slot i holds the
    transaction `row[i]` (-1 for the interleaved layout's padding slots, whose features are
    zero).  cap = slots per column (a multiple of 64, >= the layout's slot count)."""
    order = _lib.FDX_ROWS_SLOT_ORDER

    def __init__(self, cap_slots: int, device):
        self.cap = (int(cap_slots) + 63) // 64 * 64
        self.buf = torch.empty(78 * self.cap, dtype=torch.uint8, device=device)

    def columns(self, n_slots: int = None) -> dict:
        m, c = (self.cap if n_slots is None else int(n_slots)), self.cap
        i32 = self.buf[: 24 * c].view(torch.int32).view(6, c)
        f64 = self.buf[24 * c: 72 * c].view(torch.float64).view(6, c)
        row = self.buf[72 * c: 76 * c].view(torch.int32)
        fl = self.buf[76 * c: 78 * c].view(c, 2)
        return {"cust_nb": i32[0:3, :m], "term_nb": i32[3:6, :m], "cust_avg": f64[0:3, :m], "term_risk": f64[3:6, :m],
                "weekend": fl[:m, 0], "night": fl[:m, 1], "row": row[:m]}


def forest_traverse_perm(forest: "Forest", n: int, ws: torch.Tensor, out: torch.Tensor, out_perm: torch.Tensor,
                         stream=None):
    check(_lib.load().fdx_forest_traverse_perm(forest._h, n, _ptr(out), _ptr(out_perm), None, _ptr(ws), ws.numel(),
                                               _s(stream)), "fdx_forest_traverse_perm")
    return out


def forest_traverse(forest: "Forest", n: int, ws: torch.Tensor, out: torch.Tensor, stream=None):
    check(_lib.load().fdx_forest_traverse(forest._h, n, _ptr(out), None, _ptr(ws), ws.numel(), _s(stream)),
          "fdx_forest_traverse")
    return out


def forest_arrays_from_sklearn(model) -> dict:
    """sklearn DecisionTreeClassifier / RandomForestClassifier -> concatenated node arrays."""
    ests = getattr(model, "estimators_", None)
    if ests is None:
        ests = [model]
    left, right, feat, thr, ml, val, val0, off = [], [], [], [], [], [], [], [0]
    for e in ests:
        t = e.tree_
        if t.n_outputs != 1 or int(np.max(t.n_classes)) != 2:
            raise _lib.FdxUnsupported("only single-output binary classifiers are supported")
        val0.append(np.ascontiguousarray(t.value[:, 0, 0], dtype=np.float64))
        left.append(t.children_left.astype(np.int64))
        right.append(t.children_right.astype(np.int64))
        feat.append(t.feature.astype(np.int64))
        thr.append(t.threshold.astype(np.float64))
        ml.append(np.asarray(t.missing_go_to_left, dtype=np.uint8))
        val.append(np.ascontiguousarray(t.value[:, 0, 1], dtype=np.float64))
        off.append(off[-1] + t.node_count)
    return dict(left=np.concatenate(left), right=np.concatenate(right), feature=np.concatenate(feat),
                threshold=np.concatenate(thr), missing_left=np.concatenate(ml), value1=np.concatenate(val),
                value0=np.concatenate(val0), node_offsets=np.asarray(off, np.int64))
