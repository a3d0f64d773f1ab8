"""ctypes binding of libpinot_amd.so (include/pinot_amd.h).

The library is built in-tree (``python -m pinot_amd.build`` or ``__graft_entry__.build()``) and
loaded from ``pinot_amd/libpinot_amd.so``. There is no fallback: if the library is missing or a
call fails, an exception is raised.

torch (ROCm build) is imported first when available so that the process has exactly one HIP
runtime: torch ships its own ``libamdhip64.so`` with the same soname as /opt/rocm's, and the
dynamic loader then binds this library to the already-loaded copy.
"""
from __future__ import annotations

import ctypes as C
import os

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpinot_amd.so")


class PinotAmdError(RuntimeError):
    pass


class ColumnSpec(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("stored_type", C.c_int32), ("encoding", C.c_int32), ("cardinality", C.c_int32),
        ("bits_per_element", C.c_int32), ("h_fwd", C.c_void_p), ("fwd_size", C.c_size_t),
        ("h_dictionary", C.c_void_p), ("dictionary_size", C.c_size_t), ("h_inverted", C.c_void_p),
        ("inverted_size", C.c_size_t),
    ]


class PredicateSpec(C.Structure):
    _fields_ = [
        ("column", C.c_char_p), ("type", C.c_int32), ("num_values", C.c_int32),
        ("h_values_i", C.POINTER(C.c_int64)), ("h_values_d", C.POINTER(C.c_double)),
        ("h_values_s", C.POINTER(C.c_char_p)),
        ("lower_unbounded", C.c_int32), ("upper_unbounded", C.c_int32), ("lower_inclusive", C.c_int32),
        ("upper_inclusive", C.c_int32), ("lower_i", C.c_int64), ("upper_i", C.c_int64), ("lower_d", C.c_double),
        ("upper_d", C.c_double), ("lower_s", C.c_char_p), ("upper_s", C.c_char_p),
        ("use_inverted_index", C.c_int32),
    ]


# name -> (restype, argtypes); every symbol declared in include/pinot_amd.h
_P = C.c_void_p
_PP = C.POINTER(C.c_void_p)
_I64P = C.POINTER(C.c_int64)
SIGNATURES = {
    "pinot_amd_abi_version": (C.c_int, []),
    "pinot_amd_last_error": (C.c_char_p, []),
    "pinot_amd_set_device": (C.c_int, [C.c_int]),
    "pinot_amd_required_padding": (C.c_size_t, []),
    "pinot_amd_jit_selftest": (C.c_int, [C.c_int]),
    "pinot_amd_segment_create": (C.c_int, [C.c_char_p, C.c_int64, _PP]),
    "pinot_amd_segment_add_column": (C.c_int, [_P, C.POINTER(ColumnSpec)]),
    "pinot_amd_segment_destroy": (C.c_int, [_P]),
    "pinot_amd_segment_num_docs": (C.c_int64, [_P]),
    "pinot_amd_segment_device_bytes": (C.c_int64, [_P]),
    "pinot_amd_segment_column_fwd": (C.c_void_p, [_P, C.c_char_p]),
    "pinot_amd_fwd_read_dict_ids": (C.c_int, [_P, C.c_int32, C.c_int64, C.c_int64, _P, _P]),
    "pinot_amd_fwd_pack_dict_ids": (C.c_int, [_P, C.c_int64, C.c_int32, _P, _P]),
    "pinot_amd_fwd_read_raw": (C.c_int, [_P, C.c_int32, C.c_int64, C.c_int64, _P, _P]),
    "pinot_amd_bitset_and": (C.c_int, [_P, _P, _P, C.c_int64, _P]),
    "pinot_amd_bitset_or": (C.c_int, [_P, _P, _P, C.c_int64, _P]),
    "pinot_amd_bitset_not": (C.c_int, [_P, _P, C.c_int64, _P]),
    "pinot_amd_bitset_to_doc_ids": (C.c_int, [_P, C.c_int64, _P, _I64P, _P]),
    "pinot_amd_bitset_count": (C.c_int, [_P, C.c_int64, _I64P, _P]),
    "pinot_amd_query_create": (C.c_int, [_PP]),
    "pinot_amd_query_destroy": (C.c_int, [_P]),
    "pinot_amd_query_add_predicate": (C.c_int, [_P, C.c_int32, C.POINTER(PredicateSpec), C.c_int32]),
    "pinot_amd_query_add_group_by": (C.c_int, [_P, C.c_char_p]),
    "pinot_amd_query_add_aggregation": (C.c_int, [_P, C.c_int32, C.c_char_p, C.POINTER(C.c_int32)]),
    "pinot_amd_query_set_num_groups_limit": (C.c_int, [_P, C.c_int64]),
    "pinot_amd_query_set_group_key_values": (C.c_int, [_P, C.c_char_p, C.c_int32, C.c_int64, _I64P,
                                                       C.POINTER(C.c_double), C.POINTER(C.c_char_p)]),
    "pinot_amd_query_add_aggregation_expr": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_char_p, C.c_char_p,
                                                       C.POINTER(C.c_int32)]),
    "pinot_amd_result_num_groups_limit_reached": (C.c_int, [_P, C.POINTER(C.c_int32)]),
    "pinot_amd_execute": (C.c_int, [_P, _PP, C.c_int32, _P, _PP]),
    "pinot_amd_execute_filter": (C.c_int, [_P, _PP, C.c_int32, _P, _PP]),
    "pinot_amd_result_bitset": (C.c_int, [_P, C.c_int32, _PP, _I64P]),
    "pinot_amd_execute_again": (C.c_int, [_P, _P]),
    "pinot_amd_result_destroy": (C.c_int, [_P]),
    "pinot_amd_result_num_docs_matched": (C.c_int, [_P, _I64P]),
    "pinot_amd_result_num_groups": (C.c_int, [_P, _I64P]),
    "pinot_amd_result_fetch": (C.c_int, [_P, C.c_int64, _I64P, C.POINTER(C.c_double), _I64P, _I64P]),
    "pinot_amd_result_fetch_intermediate": (C.c_int, [_P, C.c_int64, C.POINTER(C.c_double), _I64P]),
    "pinot_amd_result_string_key": (C.c_char_p, [_P, C.c_int32, C.c_int64]),
    "pinot_amd_result_accumulators": (C.c_int, [_P, C.POINTER(C.c_int32), _I64P, _PP, C.POINTER(C.c_int32)]),
    "pinot_amd_result_check_word": (C.c_int, [_P, _PP]),
    "pinot_amd_selfcheck_failures": (C.c_int64, []),
    "pinot_amd_result_export_groups": (C.c_int, [_P, _P, _P, C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                                 _I64P, _P]),
    "pinot_amd_result_merge_groups": (C.c_int, [_P, _P, _P, C.c_int64, _P]),
    "pinot_amd_result_plan_timing": (C.c_char_p, [_P]),
    "pinot_amd_query_set_result_limit": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_int64]),
    "pinot_amd_query_add_order_by": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32]),
    "pinot_amd_query_set_server_options": (C.c_int, [_P, C.c_int32, C.c_int64]),
    "pinot_amd_query_set_segment_trim": (C.c_int, [_P, C.c_int64]),
    "pinot_amd_result_last_kernel_ms": (C.c_int, [_P, C.POINTER(C.c_double)]),
    "pinot_amd_result_kernel_info": (C.c_char_p, [_P]),
    "pinot_amd_result_algorithmic_bytes": (C.c_int, [_P, C.POINTER(C.c_double)]),
}

_lib = None


def lib():
    """Load libpinot_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PinotAmdError(f"{LIB_PATH} not built: run `python -m pinot_amd.build` (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().pinot_amd_last_error().decode(errors="replace")
        raise PinotAmdError(f"{what or 'pinot_amd'} failed ({rc}): {msg}")
