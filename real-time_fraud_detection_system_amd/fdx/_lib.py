"""ctypes binding of libfdx.so (include/fdx.h).  No compute happens in Python.

The library is built in-tree (``make -C real-time_fraud_detection_system_amd/csrc`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no fallback: if the
library or a GPU is missing, the calls raise.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfdx.so")

FDX_OK = 0
FDX_E_UNSUPPORTED = -3
FDX_FLAGS_NOTEBOOK = 0
FDX_FLAGS_SPARK = 1
FDX_ROWS_INPUT_ORDER = 1  # fdx_forest_prepare_grouped_rows: the featurized table by input row
FDX_ROWS_SLOT_ORDER = 2   # ... by scoring slot (coalesced; each record carries its row)
FDX_KEY_MOD, FDX_KEY_DIV, FDX_KEY_SUB = 0, 1, 2
FDX_SELECT_LATEST, FDX_SELECT_FIRST_IN_RANGE = 0, 1  # fdx_table_select
MAX_WINDOWS = 8
MAX_FEATURES = 32


class FdxError(RuntimeError):
    """A libfdx call returned a non-zero status (message from fdx_last_error())."""


class FdxUnsupported(FdxError):
    """Input the engine does not implement (FDX_E_UNSUPPORTED or a host-side check)."""


c_i32, c_i64, c_sz, P = ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p


class ForestDesc(ctypes.Structure):
    _fields_ = [
        ("n_trees", c_i32), ("n_features", c_i32),
        ("node_offsets", P), ("children_left", P), ("children_right", P), ("feature", P),
        ("threshold", P), ("missing_go_to_left", P), ("value1", P),
        ("scaler_mean", P), ("scaler_scale", P),
    ]


class SynthDesc(ctypes.Structure):
    _fields_ = [
        ("n_customers", c_i64), ("n_terminals", c_i64), ("n_days", c_i32), ("radius", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("cx", P), ("cy", P), ("mean_amount", P), ("mean_nb", P), ("tx_sorted", P), ("ty_sorted", P),
        ("t_order", P), ("range_lo", P), ("range_hi", P),
        ("comp_term", P), ("n_comp_term", c_i32), ("comp_cust", P), ("n_comp_cust", c_i32),
        ("start_ns", c_i64), ("customer_offset", c_i32),
    ]


# name -> (restype, argtypes); exactly the symbols declared in include/fdx.h
SIGNATURES = {
    "fdx_last_error": (ctypes.c_char_p, []),
    "fdx_abi_version": (ctypes.c_int, []),
    "fdx_time_flags": (ctypes.c_int, [P, c_i64, c_i32, P, P, P]),
    "fdx_customer_windows": (ctypes.c_int, [P, P, P, c_i64, c_i64, P, c_i32, P, P, P]),
    "fdx_terminal_windows_workspace_size": (c_sz, [c_i64]),
    "fdx_terminal_windows": (ctypes.c_int, [P, P, P, c_i64, c_i64, c_i64, P, c_i32, P, P, P, c_sz, P]),
    "fdx_assemble_features": (ctypes.c_int, [c_i64, c_i32, P, P, P, P, P, P, P, P, P, P, c_i64, P]),
    "fdx_customer_layout_workspace_size": (c_sz, [c_i64]),
    "fdx_customer_layout": (ctypes.c_int, [P, c_i64, P, P, P, c_i32, P, P, P, P, P, c_i64, P, P, c_sz, P]),
    "fdx_customer_layout_starts": (ctypes.c_int, [P, c_i64, P, P, P, P, c_i32, P, P, P, P, P, P, c_i64, P, P, c_sz,
                                                  P]),
    "fdx_customer_windows_walk": (ctypes.c_int, [P, P, P, P, c_i64, c_i64, c_i32, P, P, P, P]),
    "fdx_customer_windows_interleaved": (ctypes.c_int, [P, P, P, P, P, c_i64, c_i64, P, c_i32, P, P, P]),
    "fdx_exclusive_scan_u32_workspace_size": (c_sz, [c_i64]),
    "fdx_exclusive_scan_u32": (ctypes.c_int, [P, c_i64, P, P]),
    "fdx_key_segments_workspace_size": (c_sz, [c_i64]),
    "fdx_key_segments": (ctypes.c_int, [P, c_i64, c_i64, P, P, P, c_sz, P]),
    "fdx_customer_layout_plan": (ctypes.c_int, [P, c_i64, c_i32, P, P, P, P, c_sz, P]),
    "fdx_customer_layout_plan_async": (ctypes.c_int, [P, c_i64, c_i32, P, P, P, P, c_sz, P]),
    "fdx_customer_layout_fill_starts_grouped": (ctypes.c_int, [P, c_i64, P, P, P, P, c_i32, P, P, c_i64, P, P, P, P,
                                                                P]),
    "fdx_segment_latest": (ctypes.c_int, [P, P, P, c_i64, P, P]),
    "fdx_segment_first_in_range": (ctypes.c_int, [P, P, P, c_i64, c_i64, c_i64, P, P]),
    "fdx_table_select_workspace_size": (c_sz, [c_i64]),
    "fdx_table_select": (ctypes.c_int, [P, c_i64, P, P, c_i64, c_i32, c_i64, c_i64, P, P, c_sz, P]),
    "fdx_cdc_decode": (ctypes.c_int, [P, P, P, c_i64, P, P, P, P, P]),
    "fdx_dedup_latest_workspace_size": (c_sz, [c_i64]),
    "fdx_dedup_latest": (ctypes.c_int, [P, P, c_i64, P, P, P, c_sz, P]),
    "fdx_cdc_compact_workspace_size": (c_sz, [c_i64]),
    "fdx_cdc_compact": (ctypes.c_int, [P, c_i64, P, P, P, P, P, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_stream_create": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32, c_i32, P, c_i64, c_i32, c_i64, P, P]),
    "fdx_stream_reset": (ctypes.c_int, [P, P]),
    "fdx_stream_memory": (ctypes.c_int, [P, P]),
    "fdx_stream_update": (ctypes.c_int, [P, P, P, P, P, P, c_i64, P, c_i64, c_i32, P, P, P, P]),
    "fdx_stream_status": (ctypes.c_int, [P, P, P]),
    "fdx_stream_status_async": (ctypes.c_int, [P, P, P]),
    "fdx_stream_destroy": (ctypes.c_int, [P]),
    "fdx_train_test_split": (ctypes.c_int, [P, P, P, P, c_i64, c_i32, c_i64, c_i64, c_i32, c_i32, c_i32, P, P, P,
                                            c_sz, P, P]),
    "fdx_card_precision_workspace_size": (ctypes.c_size_t, [c_i32]),
    "fdx_card_precision_top_k": (ctypes.c_int, [P, P, P, P, c_i64, c_i32, P, c_i32, c_i32, c_i32, P, P, P, c_sz,
                                                P]),
    "fdx_invert_perm": (ctypes.c_int, [P, c_i64, P, P]),
    "fdx_rekey_workspace_size": (c_sz, [c_i64, c_i32]),
    "fdx_rekey": (ctypes.c_int, [P, c_i64, c_i32, c_i64, P, P, P, P, c_sz, P]),
    "fdx_rekey_payload_workspace_size": (c_sz, [c_i64, c_i32, c_i32]),
    "fdx_rekey_payload": (ctypes.c_int, [P, c_i64, c_i32, c_i64, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_rekey_payload_checked": (ctypes.c_int, [P, c_i64, c_i32, c_i64, P, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_rekey_payload_keys": (ctypes.c_int, [P, c_i64, c_i32, c_i64, P, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_segment_offsets_sorted": (ctypes.c_int, [P, c_i64, c_i64, P, P]),
    "fdx_rekey_hist0_size": (c_sz, [c_i64, c_i32]),
    "fdx_rekey_hist0": (ctypes.c_int, [P, c_i64, c_i32, c_i64, P, c_sz, P, P]),
    "fdx_rekey_payload_hist0": (ctypes.c_int, [P, c_i64, c_i32, c_i64, P, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_terminal_windows_grouped": (ctypes.c_int, [P, P, P, P, c_i64, c_i64, c_i64, P, c_i32, c_i32, P, P, P, P, P]),
    "fdx_terminal_windows_grouped_compact": (ctypes.c_int, [P, P, P, P, c_i64, c_i64, c_i64, P, c_i32, c_i32, P, P,
                                                            P]),
    "fdx_customer_layout_starts_grouped": (ctypes.c_int, [P, c_i64, P, P, P, P, c_i32, P, P, P, P, P, P, c_i64, P, P,
                                                          c_sz, P]),
    "fdx_customer_layout_grouped": (ctypes.c_int, [P, c_i64, P, P, P, c_i32, P, P, P, P, P, c_i64, P, P, c_sz, P]),
    "fdx_customer_windows_scan_workspace_size": (c_sz, [c_i64, c_i64]),
    "fdx_customer_windows_scan": (ctypes.c_int, [P, P, P, c_i64, c_i64, P, c_i32, P, P, c_i64, P, P, c_i32, P, c_sz,
                                                 P]),
    "fdx_customer_windows_scan_slots": (ctypes.c_int, [P, P, c_i64, c_i64, P, P, c_i64, c_i32, P, P, P, P, c_sz, P]),
    "fdx_argsort_i64_workspace_size": (c_sz, [c_i64]),
    "fdx_argsort_i64": (ctypes.c_int, [P, c_i64, P, P, c_sz, P]),
    "fdx_dense_ids_i64_workspace_size": (c_sz, [c_i64]),
    "fdx_dense_ids_i64": (ctypes.c_int, [P, c_i64, P, P, P, c_sz, P]),
    "fdx_is_sorted_i64": (ctypes.c_int, [P, c_i64, P, P]),
    "fdx_gather": (ctypes.c_int, [P, c_i32, P, c_i64, P, P]),
    "fdx_scatter": (ctypes.c_int, [P, c_i32, P, c_i64, P, P]),
    "fdx_key_map": (ctypes.c_int, [P, c_i64, c_i32, c_i32, P, P]),
    "fdx_count_out_of_range": (ctypes.c_int, [P, c_i64, c_i32, c_i32, P, P]),
    "fdx_exchange_pack": (ctypes.c_int, [P, P, P, P, c_i64, P, P]),
    "fdx_exchange_unpack": (ctypes.c_int, [P, c_i64, c_i32, P, P, P, P]),
    "fdx_reply_assemble": (ctypes.c_int, [P, P, c_i64, c_i32, P, c_i64, c_i32, P]),
    "fdx_standard_scale": (ctypes.c_int, [P, c_i64, c_i32, c_i64, c_i64, P, P, P, c_i64, c_i64, P]),
    "fdx_forest_create": (ctypes.c_int, [ctypes.POINTER(ForestDesc), ctypes.POINTER(P), P]),
    "fdx_forest_pack": (ctypes.c_int, [ctypes.POINTER(ForestDesc), P, P, P]),
    "fdx_forest_rank_layout_size": (ctypes.c_int, [ctypes.POINTER(ForestDesc), P, P]),
    "fdx_forest_pack_rank": (ctypes.c_int, [ctypes.POINTER(ForestDesc), P, P, P, P, P, P, P, P]),
    "fdx_forest_rank_layout_size2": (ctypes.c_int, [ctypes.POINTER(ForestDesc), c_i32, P, P, P]),
    "fdx_forest_pack_rank2": (ctypes.c_int, [ctypes.POINTER(ForestDesc), c_i32, P, P, P, P, P, P, P, P, P, P]),
    "fdx_forest_search_trees": (ctypes.c_int, [ctypes.POINTER(ForestDesc), P, c_i64, P, P, P]),
    "fdx_forest_layout": (ctypes.c_int, [P, P, P]),
    "fdx_forest_destroy": (ctypes.c_int, [P]),
    "fdx_synth_workspace_size": (c_sz, [ctypes.POINTER(SynthDesc), c_i64]),
    "fdx_synth_plan": (ctypes.c_int, [ctypes.POINTER(SynthDesc), P, c_sz, P, P]),
    "fdx_synth_fill": (ctypes.c_int, [ctypes.POINTER(SynthDesc), c_i64, P, c_sz, P, P, P, P, P, P, P, P]),
    "fdx_forest_info": (ctypes.c_int, [P, P, P, P, P]),
    "fdx_forest_traverse_launches": (ctypes.c_int, [P, ctypes.c_int64, ctypes.c_int32, P]),
    "fdx_forest_workspace_size": (c_sz, [P, c_i64]),
    "fdx_forest_workspace_size_max": (ctypes.c_size_t, [P, c_i64]),
    "fdx_forest_predict": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, P, P, P, c_sz, P]),
    "fdx_forest_prepare": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, P, c_sz, P]),
    "fdx_forest_traverse": (ctypes.c_int, [P, c_i64, P, P, P, c_sz, P]),
    "fdx_forest_prepare_features": (ctypes.c_int, [P, c_i64, c_i32, P, P, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_forest_clear_flag": (ctypes.c_int, [P, c_i64, P, c_sz, P]),
    "fdx_forest_prepare_grouped": (ctypes.c_int, [P, c_i64, c_i32, c_i32, c_i32, P, P, P, P, P, P, P, P, c_sz, P]),
    "fdx_forest_prepare_grouped_rows": (ctypes.c_int, [P, c_i64, c_i32, c_i32, c_i32, P, P, P, P, P, P, P, P, c_i64,
                                                       c_i32, P, c_sz, P]),
    "fdx_forest_traverse_perm": (ctypes.c_int, [P, c_i64, P, P, P, P, c_sz, P]),
    "fdx_forest_set_variant": (ctypes.c_int, [P, c_i32]),
    "fdx_forest_get_variant": (ctypes.c_int, [P, P]),
    "fdx_forest_set_range_rows": (ctypes.c_int, [P, ctypes.c_int64]),
    "fdx_forest_prepare_reply": (ctypes.c_int, [P, P, P, c_i64, c_i32, c_i32, P, c_sz, P]),
}

_lib = None


def load():
    """Load libfdx.so (raises FdxError when it is missing -- there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FdxError(f"{LIB_PATH} not built: run `make -C real-time_fraud_detection_system_amd/csrc` "
                           "(or __graft_entry__.build()); fdx has no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.fdx_abi_version() != 2:
            raise FdxError("libfdx ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != FDX_OK:
        msg = load().fdx_last_error().decode(errors="replace")
        cls = FdxUnsupported if rc == -3 else FdxError
        raise cls(f"{what or 'fdx'} failed ({rc}): {msg}")
