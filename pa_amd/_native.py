"""ctypes binding of libstrawboat_gpu.so (include/strawboat_gpu.h).

The product path: every decode runs the HIP kernels in the in-tree
libstrawboat_gpu.so.  If the library is missing or no GPU is visible the
calls raise; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PA_AMD_LIB") or os.path.join(_HERE, "libstrawboat_gpu.so")

# sb_status
OK, E_OUT_OF_SPEC, E_NYI, E_IO, E_CODEC, E_DEVICE, E_ARG = 0, 1, 2, 3, 4, 5, 6

# sb_physical_type
INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64, FLOAT32, FLOAT64 = range(1, 11)
BOOLEAN = 15

EXPORTED = [
    "sb_ctx_create", "sb_ctx_destroy", "sb_ctx_set_stream", "sb_ctx_stream", "sb_ctx_device", "sb_sync", "sb_last_error",
    "sb_status_str", "sb_plan_column", "sb_plan_destroy", "sb_plan_num_rows", "sb_plan_num_pages",
    "sb_decode_planned", "sb_plan_status", "sb_decode_column", "sb_plan_last_kernel_ms", "sb_plan_enable_timing",
    "sb_decompress_values", "sb_read_meta", "sb_encode_page", "sb_encode_column", "sb_page_seed",
    "sb_write_footer", "sb_free", "sb_encode_binary_column", "sb_plan_values_bytes", "sb_decode_binary_planned",
    "sb_encode_list_column", "sb_plan_list_column", "sb_plan_num_leaves", "sb_decode_list_planned",
    "sb_encode_device_bound", "sb_encode_column_device", "sb_lz4_compress_host", "sb_snappy_compress_host", "sb_zstd_compress_host",
    "sb_encode_binary_device_bound", "sb_encode_binary_column_device", "sb_plan_nested_column",
    "sb_plan_nested_count", "sb_decode_nested_planned", "sb_parse_schema", "sb_file_open", "sb_file_close",
    "sb_file_last_error", "sb_file_num_columns", "sb_file_column", "sb_file_schema", "sb_file_upload",
    "sb_decode_page_validity", "sb_decode_page_levels", "sb_plan_column_at",
    "sb_encode_list_device_bound", "sb_encode_list_column_device", "sb_encode_nested_column",
]

MAX_NEST = 4


class StrawboatError(RuntimeError):
    """arrow2::error::Error analogue: .status is the sb_status code."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"[{status}] {msg}")
        self.status = status


class PageMetaC(ctypes.Structure):
    _fields_ = [("length", ctypes.c_uint64), ("num_values", ctypes.c_uint64)]


class ColumnDescC(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("nullable", ctypes.c_int32)]


class WriteOptionsC(ctypes.Structure):
    _fields_ = [
        ("default_codec", ctypes.c_int32),
        ("has_ratio", ctypes.c_int32),
        ("ratio", ctypes.c_double),
        ("forbidden_mask", ctypes.c_uint32),
        ("forced_codec", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
    ]


class LeafInfoC(ctypes.Structure):
    """sb_leaf_info"""
    _fields_ = [("name", ctypes.c_char * 64), ("arrow_type", ctypes.c_int32), ("physical_type", ctypes.c_int32),
                ("nullable", ctypes.c_int32), ("depth", ctypes.c_int32), ("list_nullable", ctypes.c_int32 * MAX_NEST),
                ("large_list", ctypes.c_int32 * MAX_NEST), ("flags", ctypes.c_uint32), ("top_field", ctypes.c_int32),
                ("struct_mask", ctypes.c_uint32), ("map_mask", ctypes.c_uint32), ("nest_id", ctypes.c_int32 * MAX_NEST)]


class PrimitiveOutC(ctypes.Structure):
    _fields_ = [("d_values", ctypes.c_void_p), ("d_validity", ctypes.c_void_p)]


def build(force: bool = False) -> str:
    """Compile the HIP library for gfx950 in-tree (make -C pa_amd)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `make -C pa_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
    PP = ctypes.POINTER(ctypes.c_void_p)
    L.sb_ctx_create.argtypes = [ctypes.c_int, PP]
    L.sb_ctx_create.restype = I32
    L.sb_ctx_destroy.argtypes = [P]
    L.sb_ctx_destroy.restype = None
    L.sb_ctx_set_stream.argtypes = [P, P]
    L.sb_ctx_set_stream.restype = I32
    L.sb_ctx_stream.argtypes = [P]
    L.sb_ctx_stream.restype = P
    L.sb_ctx_device.argtypes = [P]
    L.sb_ctx_device.restype = I32
    L.sb_sync.argtypes = [P]
    L.sb_sync.restype = I32
    L.sb_last_error.argtypes = [P]
    L.sb_last_error.restype = ctypes.c_char_p
    L.sb_status_str.argtypes = [ctypes.c_int]
    L.sb_status_str.restype = ctypes.c_char_p
    L.sb_plan_column.argtypes = [P, ctypes.POINTER(ColumnDescC), P, U64, ctypes.POINTER(PageMetaC), U64, PP]
    L.sb_plan_column.restype = I32
    L.sb_plan_column_at.argtypes = [P, ctypes.POINTER(ColumnDescC), P, U64, ctypes.POINTER(PageMetaC), U64, P, PP]
    L.sb_plan_column_at.restype = I32
    L.sb_plan_destroy.argtypes = [P]
    L.sb_plan_destroy.restype = None
    L.sb_plan_num_rows.argtypes = [P]
    L.sb_plan_num_rows.restype = U64
    L.sb_plan_num_pages.argtypes = [P]
    L.sb_plan_num_pages.restype = U64
    L.sb_decode_planned.argtypes = [P, P, ctypes.POINTER(PrimitiveOutC)]
    L.sb_decode_planned.restype = I32
    L.sb_plan_status.argtypes = [P, P, ctypes.POINTER(ctypes.c_int64)]
    L.sb_plan_status.restype = I32
    L.sb_decode_column.argtypes = [P, ctypes.POINTER(ColumnDescC), P, U64, ctypes.POINTER(PageMetaC), U64,
                                   ctypes.POINTER(PrimitiveOutC)]
    L.sb_decode_column.restype = I32
    L.sb_plan_enable_timing.argtypes = [P, I32]
    L.sb_plan_enable_timing.restype = I32
    L.sb_plan_last_kernel_ms.argtypes = [P, P, ctypes.POINTER(ctypes.c_float)]
    L.sb_plan_last_kernel_ms.restype = I32
    L.sb_decompress_values.argtypes = [P, I32, P, U64, U64, P]
    L.sb_decompress_values.restype = I32
    L.sb_decode_page_validity.argtypes = [P, P, U64, U64, P, U64, ctypes.POINTER(U64)]
    L.sb_decode_page_validity.restype = I32
    L.sb_decode_page_levels.argtypes = [P, P, U64, U64, ctypes.c_uint32, ctypes.c_uint32, P, P,
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(U64)]
    L.sb_decode_page_levels.restype = I32
    L.sb_read_meta.argtypes = [P, U64, P, P, U64, P, U64, ctypes.POINTER(U64), ctypes.POINTER(U64)]
    L.sb_read_meta.restype = I32
    PU8 = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))
    L.sb_encode_page.argtypes = [I32, P, P, U64, I32, ctypes.POINTER(WriteOptionsC), U64, PU8, ctypes.POINTER(U64)]
    L.sb_encode_page.restype = I32
    L.sb_encode_column.argtypes = [I32, P, P, U64, I32, ctypes.POINTER(WriteOptionsC), U64, I32, PU8,
                                   ctypes.POINTER(U64), ctypes.POINTER(ctypes.POINTER(PageMetaC)), ctypes.POINTER(U64)]
    L.sb_encode_column.restype = I32
    L.sb_encode_device_bound.argtypes = [I32, U64, I32, U64]
    L.sb_encode_device_bound.restype = U64
    L.sb_encode_column_device.argtypes = [P, I32, P, P, U64, I32, ctypes.POINTER(WriteOptionsC), U64, P, U64,
                                          ctypes.POINTER(U64), ctypes.POINTER(PageMetaC), U64, ctypes.POINTER(U64)]
    L.sb_encode_column_device.restype = I32
    L.sb_encode_list_device_bound.argtypes = [I32, U64, U64, I32, U64]
    L.sb_encode_list_device_bound.restype = U64
    L.sb_encode_list_column_device.argtypes = [P, I32, P, P, I32, P, P, I32, U64, ctypes.POINTER(WriteOptionsC), U64,
                                               P, U64, ctypes.POINTER(U64), ctypes.POINTER(PageMetaC), U64,
                                               ctypes.POINTER(U64)]
    L.sb_encode_list_column_device.restype = I32
    L.sb_page_seed.argtypes = [U64, U64]
    L.sb_page_seed.restype = U64
    L.sb_write_footer.argtypes = [P, U64, P, P, U64, P, PU8, ctypes.POINTER(U64)]
    L.sb_write_footer.restype = I32
    L.sb_free.argtypes = [P]
    L.sb_free.restype = None
    L.sb_parse_schema.argtypes = [P, U64, ctypes.POINTER(LeafInfoC), U64, ctypes.POINTER(U64), ctypes.POINTER(U64)]
    L.sb_parse_schema.restype = I32
    L.sb_file_open.argtypes = [ctypes.c_char_p, PP]
    L.sb_file_open.restype = I32
    L.sb_file_close.argtypes = [P]
    L.sb_file_close.restype = None
    L.sb_file_last_error.argtypes = [P]
    L.sb_file_last_error.restype = ctypes.c_char_p
    L.sb_file_num_columns.argtypes = [P]
    L.sb_file_num_columns.restype = U64
    L.sb_file_column.argtypes = [P, U64, ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.POINTER(U64),
                                 ctypes.POINTER(ctypes.POINTER(PageMetaC))]
    L.sb_file_column.restype = I32
    L.sb_file_schema.argtypes = [P, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(U64)]
    L.sb_file_schema.restype = I32
    L.sb_file_upload.argtypes = [P, P, U64, U64, P]
    L.sb_file_upload.restype = I32
    _lib = L
    return L
