"""Host-side decoders of the terminal count records (test helpers: the product's kernels read
these formats themselves).  Plain numpy, so tests compare the device records on the host."""
import numpy as np


def compact_records_unpack(rec, n: int) -> np.ndarray:
    """terminal_windows_compact's array (int64, 5n words: a 16-byte pair per row + the overflow
    area) -> the [n, 3] int64 count records (NB | FRAUD << 32)."""
    rec = np.asarray(rec.cpu().numpy() if hasattr(rec, "cpu") else rec, dtype=np.int64)
    pair = rec[: 2 * n].reshape(n, 2)
    lo, hi = pair[:, 0], pair[:, 1]
    m = (1 << 21) - 1
    out = np.stack([((lo >> (21 * w)) & m) | (((hi >> (21 * w)) & m) << 32) for w in range(3)], axis=1)
    esc = lo < 0
    if esc.any():
        off = lo[esc] & ((1 << 63) - 1)
        out[esc] = np.stack([rec[off + w] for w in range(3)], axis=1)
    return out


def unpack_term_records(rec):
    """Count records [n, W] -> (nb int32 [W, n], risk float64 [W, n]) with the kernels' IEEE
    division (NB_FRAUD / NB_TX, 0 where NB_TX = 0)."""
    w = np.asarray(rec.cpu().numpy() if hasattr(rec, "cpu") else rec, dtype=np.int64).T
    nb = (w & 0xFFFFFFFF).astype(np.int32)
    fr = (w >> 32) & 0xFFFFFFFF
    with np.errstate(invalid="ignore", divide="ignore"):
        risk = np.where(nb > 0, fr.astype(np.float64) / np.maximum(nb, 1).astype(np.float64), 0.0)
    return nb, risk
