"""ctypes binding of libfury_row.so (include/fury_row.h).

The library is built in-tree (``fury_amd/libfury_row.so``, see fury_amd/csrc/Makefile and
``__graft_entry__.build()``).  There is no fallback: if the library is missing or fails to load,
importing this module raises, so no code path silently runs on the CPU.
"""
from __future__ import annotations

import ctypes
import os

# torch first: its bundled libamdhip64.so.7 must be the HIP runtime our library binds to, so
# that torch streams/allocations and our launches share one runtime.
import torch  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
# FURY_ROW_LIB: alternative in-tree build of the same library (kernel-variant A/B experiments)
LIB_PATH = os.environ.get("FURY_ROW_LIB") or os.path.join(HERE, "libfury_row.so")


class FuryField(ctypes.Structure):
    pass


FuryField._fields_ = [("name", ctypes.c_char_p), ("type_id", ctypes.c_int32),
                      ("nullable", ctypes.c_int32), ("num_children", ctypes.c_int32),
                      ("children", ctypes.POINTER(FuryField))]


class FuryColumn(ctypes.Structure):
    pass


FuryColumn._fields_ = [("values", ctypes.c_void_p), ("validity", ctypes.c_void_p),
                       ("offsets", ctypes.c_void_p), ("capacity", ctypes.c_int64),
                       ("child", ctypes.POINTER(FuryColumn))]


class FurySchemaInfo(ctypes.Structure):
    _fields_ = [("num_fields", ctypes.c_int32), ("bitmap_bytes", ctypes.c_int32),
                ("fixed_size", ctypes.c_int32), ("is_fixed", ctypes.c_int32),
                ("schema_hash", ctypes.c_int64)]


# Exported symbols with their signatures (kept in sync with include/fury_row.h; the CPU test
# suite checks the header and this table agree).
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
SIGNATURES = {
    "fury_abi_version": (_I32, []),
    "fury_last_error": (ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t]),
    "fury_type_width": (_I32, [_I32]),
    "fury_sort_bean_fields": (ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), _I32,
                                             ctypes.POINTER(_I32)]),
    "fury_lower_camel_to_lower_underscore": (_I32, [ctypes.c_char_p, ctypes.c_char_p,
                                                    ctypes.c_size_t]),
    "fury_schema_create": (ctypes.c_int, [ctypes.POINTER(FuryField), _I32, ctypes.POINTER(_P)]),
    "fury_collection_schema_create": (ctypes.c_int, [ctypes.POINTER(FuryField), ctypes.POINTER(_P)]),
    "fury_schema_destroy": (None, [_P]),
    "fury_schema_get_info": (ctypes.c_int, [_P, ctypes.POINTER(FurySchemaInfo)]),
    "fury_row_measure": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I64, _P, _P]),
    "fury_row_encode": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I64, _P, _P, _P]),
    "fury_row_encode_measured": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I64, _P, _P, _I64,
                                                _P]),
    "fury_row_decode_measure": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(FuryColumn),
                                               _P]),
    "fury_row_decode": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(FuryColumn), _P]),
    "fury_rows_to_arrow": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(FuryColumn), _P]),
    "fury_schema_num_nodes": (_I32, [_P]),
    "fury_decode_prepare": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(_I64),
                                           ctypes.POINTER(_I64), ctypes.POINTER(_P), _P]),
    "fury_decode_execute": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I32, _P]),
    "fury_decode_plan_destroy": (None, [_P]),
    "fury_device_status": (ctypes.c_int, [_P]),
    "fury_stream_release": (ctypes.c_int, [_P]),
    "fury_trim_workspace": (ctypes.c_int, [_I32]),
    "fury_set_tuning": (ctypes.c_int, [ctypes.c_char_p, _I32]),
    "fury_get_tuning": (_I32, [ctypes.c_char_p]),
    "fury_arrow_append": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I64,
                                         ctypes.POINTER(FuryColumn), _I64, _P]),
    "fury_frame_rows": (ctypes.c_int, [_P, _P, _P, _I64, _P, _P, _P]),
    "fury_unframe_rows": (ctypes.c_int, [_P, _P, _I64, _I64, _P, _P, _P]),
    "fury_host_alloc": (ctypes.c_int, [_I64, ctypes.POINTER(ctypes.c_void_p)]),
    "fury_host_free": (ctypes.c_int, [_P]),
    "fury_host_register": (ctypes.c_int, [_P, _I64]),
    "fury_host_unregister": (ctypes.c_int, [_P]),
    "fury_row_encode_host": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I64, _P, _I64, _P,
                                            ctypes.POINTER(_I64), _I32]),
    "fury_row_decode_host": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(FuryColumn), _I32]),
    "fury_decode_host_prepare": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(_I64),
                                                ctypes.POINTER(_I64), ctypes.POINTER(_P), _I32]),
    "fury_decode_host_execute": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn)]),
    "fury_jni_exception_class": (ctypes.c_char_p, [ctypes.c_int]),
    "fury_jni_schema_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I32),
                                              _I32, _I32, ctypes.POINTER(_P)]),
    "fury_jni_encode_host": (ctypes.c_int, [_P, ctypes.POINTER(_I64), _I64, _I64, _P, _I64, _P,
                                            ctypes.POINTER(_I64), _I32]),
    "fury_jni_decode_host": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(_I64), _I64, _I32]),
    "fury_jni_decode_host_prepare": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(_I64), _I64,
                                                    ctypes.POINTER(_P), _I32]),
    "fury_jni_decode_host_execute": (ctypes.c_int, [_P, _P, ctypes.POINTER(_I64), _I64]),
    "fury_hbm_copy": (ctypes.c_int, [_P, _P, _I64, _P]),
    "fury_arrow_ipc_schema": (ctypes.c_int, [_P, _P, _I64, ctypes.POINTER(_I64)]),
    "fury_arrow_ipc_record_batch": (ctypes.c_int, [_P, ctypes.POINTER(FuryColumn), _I64, _P, _I64,
                                                   ctypes.POINTER(_I64), _P]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("FURY_ROW_LIB") and not hasattr(L, name):
                continue          # an older build for A/B: entry points it predates stay unbound
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(4096)
    lib().fury_last_error(buf, len(buf))
    return buf.value.decode("utf-8", "replace")
