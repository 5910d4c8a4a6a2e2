"""ctypes wrapper over oracle/_build/libsb_oracle.so.

TEST INFRASTRUCTURE ONLY: the CPU restatement of the strawboat (b41sh/pa)
codec path used as the parity checker and as bench.py's cpu_baseline leg.
The product package (pa_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libsb_oracle.so")

# codec ids (compression/mod.rs:64-82)
NONE, LZ4, ZSTD, SNAPPY = 0, 1, 2, 3
RLE, DICT, ONE_VALUE, FREQ, BITPACKING, DELTA_BITPACKING, PATAS = 10, 11, 12, 13, 14, 15, 16


class OracleError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: oracle status {code}")
        self.code = code


class _Buf(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("len", ctypes.c_size_t), ("cap", ctypes.c_size_t)]


class WriteOptions(ctypes.Structure):
    """write::WriteOptions (write/common.rs:37-45) + forced codec + sampler seed."""

    _fields_ = [
        ("default_codec", ctypes.c_int32),
        ("has_ratio", ctypes.c_int32),
        ("ratio", ctypes.c_double),
        ("forbidden_mask", ctypes.c_uint32),
        ("forced_codec", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
    ]

    @classmethod
    def make(cls, default_codec=NONE, ratio=None, forbidden=(), forced=-1, seed=42):
        m = 0
        for c in forbidden:
            m |= 1 << c
        return cls(default_codec, ratio is not None, float(ratio or 0.0), m, forced, seed)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        PS = ctypes.POINTER(ctypes.c_size_t)
        L.orc_buf_free.argtypes = [ctypes.POINTER(_Buf)]
        L.orc_bp4x_num_bits.argtypes = [P]
        L.orc_bp4x_num_bits.restype = ctypes.c_uint32
        for f in ("orc_bp4x_pack", "orc_bp4x_unpack"):
            getattr(L, f).argtypes = [P, ctypes.c_uint32, P]
            getattr(L, f).restype = S
        for f in ("orc_bp4x_pack_sorted", "orc_bp4x_unpack_sorted"):
            getattr(L, f).argtypes = [ctypes.c_uint32, P, ctypes.c_uint32, P]
            getattr(L, f).restype = S
        for f in ("orc_decompress_integer", "orc_decompress_double"):
            getattr(L, f).argtypes = [P, S, PS, I, S, P]
            getattr(L, f).restype = I
        L.orc_compress_integer.argtypes = [P, P, S, I, I, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf)]
        L.orc_compress_double.argtypes = [P, P, S, I, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf)]
        L.orc_patas_pack.argtypes = [ctypes.c_uint32] * 3
        L.orc_patas_pack.restype = ctypes.c_uint16
        L.orc_patas_unpack.argtypes = [ctypes.c_uint16] + [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.orc_read_validity.argtypes = [P, S, PS, S, P]
        L.orc_write_validity.argtypes = [P, S, ctypes.POINTER(_Buf)]
        L.orc_read_flat_page.argtypes = [P, S, S, I, I, I, P, P]
        L.orc_write_flat_page.argtypes = [P, P, S, I, I, I, I, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf)]
        L.orc_read_column.argtypes = [P, S, P, S, I, I, I, P, P]
        L.orc_roaring_decode.argtypes = [P, S, P, S, PS]
        L.orc_roaring_encode.argtypes = [P, S, ctypes.POINTER(_Buf)]
        L.orc_hybrid_decode.argtypes = [P, S, ctypes.c_uint32, S, P]
        L.orc_common_decompress.argtypes = [I, P, S, P, S]
        L.orc_common_compress.argtypes = [I, P, S, ctypes.POINTER(_Buf)]
        L.orc_compress_boolean.argtypes = [P, S, P, S, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf)]
        L.orc_decompress_boolean.argtypes = [P, S, PS, S, P]
        L.orc_write_bool_page.argtypes = [P, S, P, S, I, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf)]
        L.orc_read_bool_page.argtypes = [P, S, S, I, P, P]
        L.orc_read_bool_column.argtypes = [P, S, P, S, I, P, P]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _take(buf: _Buf) -> bytes:
    out = ctypes.string_at(buf.data, buf.len) if buf.len else b""
    lib().orc_buf_free(ctypes.byref(buf))
    return out


def _check(rc, what):
    if rc:
        raise OracleError(rc, what)


def _bytes_arr(b: bytes) -> np.ndarray:
    return np.frombuffer(b, dtype=np.uint8).copy() if b else np.zeros(1, np.uint8)


# ---- BitPacker4x ----------------------------------------------------------
def bp4x_num_bits(block: np.ndarray) -> int:
    block = np.ascontiguousarray(block, dtype=np.uint32)
    return lib().orc_bp4x_num_bits(_ptr(block))


def bp4x_pack(block: np.ndarray, b: int, sorted_initial=None) -> bytes:
    block = np.ascontiguousarray(block, dtype=np.uint32)
    out = np.zeros(512, np.uint8)
    if sorted_initial is None:
        n = lib().orc_bp4x_pack(_ptr(block), b, _ptr(out))
    else:
        n = lib().orc_bp4x_pack_sorted(sorted_initial, _ptr(block), b, _ptr(out))
    return out[:n].tobytes()


def bp4x_unpack(data: bytes, b: int, sorted_initial=None) -> np.ndarray:
    src = np.zeros(512 + 16, np.uint8)
    src[: len(data)] = np.frombuffer(data, np.uint8)
    out = np.zeros(128, np.uint32)
    if sorted_initial is None:
        lib().orc_bp4x_unpack(_ptr(src), b, _ptr(out))
    else:
        lib().orc_bp4x_unpack_sorted(sorted_initial, _ptr(src), b, _ptr(out))
    return out


# ---- value streams ----------------------------------------------------------
def compress(values: np.ndarray, validity=None, opts: WriteOptions | None = None) -> bytes:
    """compress_integer / compress_double on one page's values."""
    values = np.ascontiguousarray(values)
    opts = opts or WriteOptions.make()
    buf = _Buf()
    vb = None if validity is None else np.packbits(np.asarray(validity, bool), bitorder="little")
    if values.dtype.kind == "f":
        rc = lib().orc_compress_double(_ptr(values), _ptr(vb), len(values), values.itemsize, ctypes.byref(opts), ctypes.byref(buf))
    else:
        rc = lib().orc_compress_integer(
            _ptr(values), _ptr(vb), len(values), values.itemsize, int(values.dtype.kind == "i"), ctypes.byref(opts), ctypes.byref(buf)
        )
    data = _take(buf)
    _check(rc, "compress")
    return data


def decompress(data: bytes, dtype, length: int, pos: int = 0):
    """decompress_integer / decompress_double; returns (values, new_pos)."""
    dtype = np.dtype(dtype)
    src = _bytes_arr(data)
    out = np.zeros(max(length, 1), dtype)
    p = ctypes.c_size_t(pos)
    f = lib().orc_decompress_double if dtype.kind == "f" else lib().orc_decompress_integer
    rc = f(_ptr(src), len(data), ctypes.byref(p), dtype.itemsize, length, _ptr(out))
    _check(rc, "decompress")
    return out[:length], p.value


def write_validity(validity) -> bytes:
    v = np.packbits(np.asarray(validity, bool), bitorder="little")
    buf = _Buf()
    _check(lib().orc_write_validity(_ptr(v), len(validity), ctypes.byref(buf)), "write_validity")
    return _take(buf)


def read_validity(data: bytes, length: int, pos: int = 0):
    src = _bytes_arr(data)
    out = np.zeros((length + 7) // 8 + 1, np.uint8)
    p = ctypes.c_size_t(pos)
    _check(lib().orc_read_validity(_ptr(src), len(data), ctypes.byref(p), length, _ptr(out)), "read_validity")
    return np.unpackbits(out, bitorder="little")[:length].astype(bool), p.value


def write_page(values: np.ndarray, validity=None, nullable=False, opts: WriteOptions | None = None) -> bytes:
    """One flat page as serialize::write_simple emits it (serialize.rs:52-132)."""
    values = np.ascontiguousarray(values)
    opts = opts or WriteOptions.make()
    vb = None
    if validity is not None:
        vb = np.packbits(np.asarray(validity, bool), bitorder="little")
    buf = _Buf()
    kind = 1 if values.dtype.kind == "f" else 0
    rc = lib().orc_write_flat_page(
        _ptr(values), _ptr(vb), len(values), kind, values.itemsize, int(values.dtype.kind == "i"), int(nullable), ctypes.byref(opts), ctypes.byref(buf)
    )
    data = _take(buf)
    _check(rc, "write_page")
    return data


def read_page(page: bytes, num_values: int, dtype, nullable=False):
    """IntegerIter / DoubleIter::deserialize on one page -> (values, validity|None)."""
    dtype = np.dtype(dtype)
    src = _bytes_arr(page)
    out = np.zeros(max(num_values, 1), dtype)
    bits = np.zeros((num_values + 7) // 8 + 1, np.uint8)
    kind = 1 if dtype.kind == "f" else 0
    rc = lib().orc_read_flat_page(_ptr(src), len(page), num_values, kind, dtype.itemsize, int(nullable), _ptr(out), _ptr(bits))
    _check(rc, "read_page")
    validity = np.unpackbits(bits, bitorder="little")[:num_values].astype(bool) if nullable else None
    return out[:num_values], validity


def roaring_encode(positions) -> bytes:
    p = np.ascontiguousarray(positions, dtype=np.uint32)
    buf = _Buf()
    _check(lib().orc_roaring_encode(_ptr(p), len(p), ctypes.byref(buf)), "roaring_encode")
    return _take(buf)


def roaring_decode(data: bytes) -> np.ndarray:
    src = _bytes_arr(data)
    cnt = ctypes.c_size_t(0)
    _check(lib().orc_roaring_decode(_ptr(src), len(data), None, 0, ctypes.byref(cnt)), "roaring_decode")
    out = np.zeros(max(cnt.value, 1), np.uint32)
    _check(lib().orc_roaring_decode(_ptr(src), len(data), _ptr(out), cnt.value, ctypes.byref(cnt)), "roaring_decode")
    return out[: cnt.value]


def hybrid_decode(data: bytes, bit_width: int, n: int) -> np.ndarray:
    src = _bytes_arr(data)
    out = np.zeros(max(n, 1), np.uint32)
    _check(lib().orc_hybrid_decode(_ptr(src), len(data), bit_width, n, _ptr(out)), "hybrid_decode")
    return out[:n]


def common_compress(codec: int, data: bytes) -> bytes:
    src = _bytes_arr(data)
    buf = _Buf()
    rc = lib().orc_common_compress(codec, _ptr(src), len(data), ctypes.byref(buf))
    out = _take(buf)
    _check(rc, "common_compress")
    return out


def common_decompress(codec: int, data: bytes, out_len: int) -> bytes:
    src = _bytes_arr(data)
    out = np.zeros(max(out_len, 1), np.uint8)
    _check(lib().orc_common_decompress(codec, _ptr(src), len(data), _ptr(out), out_len), "common_decompress")
    return out[:out_len].tobytes()


def patas_pack(r, s, t) -> int:
    return lib().orc_patas_pack(r, s, t)


def patas_unpack(p: int):
    a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    lib().orc_patas_unpack(p, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value, b.value, c.value


def page_codec(page: bytes, nullable: bool) -> int:
    """Codec byte of a flat page's value stream (after the validity prefix)."""
    pos = 0
    if nullable:
        pos = 4 + int.from_bytes(page[:4], "little")
    return page[pos]


def read_column(chunk: bytes, metas, dtype, nullable=False):
    """read_integer / read_double over a whole column chunk (one C call)."""
    dtype = np.dtype(dtype)
    n = sum(int(nv) for _, nv in metas)
    m = np.asarray([(int(l), int(nv)) for l, nv in metas], dtype=np.uint64).reshape(-1)
    src = np.frombuffer(chunk, dtype=np.uint8)
    out = np.zeros(max(n, 1), dtype)
    bits = np.zeros((n + 7) // 8 + 1, np.uint8)
    kind = 1 if dtype.kind == "f" else 0
    rc = lib().orc_read_column(_ptr(src), len(chunk), _ptr(m), len(metas), kind, dtype.itemsize, int(nullable), _ptr(out), _ptr(bits))
    _check(rc, "read_column")
    return out[:n], (np.unpackbits(bits, bitorder="little")[:n].astype(bool) if nullable else None)


# ---- binary / utf8 ------------------------------------------------------------
class _BinVec(ctypes.Structure):
    _fields_ = [("offsets", ctypes.POINTER(ctypes.c_int64)), ("n_off", ctypes.c_size_t), ("cap_off", ctypes.c_size_t),
                ("values", ctypes.POINTER(ctypes.c_uint8)), ("n_val", ctypes.c_size_t), ("cap_val", ctypes.c_size_t)]


def _bin_lib():
    L = lib()
    if not getattr(L, "_bin_ready", False):
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.orc_binvec_free.argtypes = [ctypes.POINTER(_BinVec)]
        L.orc_read_binary_page.argtypes = [P, S, S, I, I, ctypes.POINTER(_BinVec), P]
        L.orc_write_binary_page.argtypes = [P, P, P, S, I, I, ctypes.c_uint64, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf)]
        L._bin_ready = True
    return L


def strings_to_arrow(strings):
    """list of bytes -> (values bytes, int64 offsets n+1)."""
    offs = np.zeros(len(strings) + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in strings])
    return b"".join(strings), offs


def write_binary_page(values: bytes, offsets: np.ndarray, validity=None, nullable=False, opts=None,
                      offset_width=4, parent_values_len=None) -> bytes:
    """write_simple for Binary/Utf8 (serialize.rs:64-110) over rows
    offsets[0..n]; parent_values_len = the array's whole values buffer."""
    L = _bin_lib()
    opts = opts or WriteOptions.make()
    n = len(offsets) - 1
    offs = np.ascontiguousarray(offsets, np.int64)
    vals = np.frombuffer(values, np.uint8) if values else np.zeros(1, np.uint8)
    vb = None if validity is None else np.packbits(np.asarray(validity, bool), bitorder="little")
    buf = _Buf()
    pl = len(values) if parent_values_len is None else parent_values_len
    rc = L.orc_write_binary_page(_ptr(vals), _ptr(offs), _ptr(vb), n, offset_width, int(nullable), pl, ctypes.byref(opts), ctypes.byref(buf))
    data = _take(buf)
    _check(rc, "write_binary_page")
    return data


def read_binary_column(chunk: bytes, metas, nullable=False, offset_width=4):
    """read_binary (read/array/binary.rs:223-265): pages appended -> (offsets
    int64 array of n+1, values bytes, validity|None)."""
    L = _bin_lib()
    src = np.frombuffer(chunk, np.uint8) if chunk else np.zeros(1, np.uint8)
    bv = _BinVec()
    valid = []
    pos = 0
    try:
        for length, nv in metas:
            bits = np.zeros((nv + 7) // 8 + 1, np.uint8)
            page = src[pos:pos + length]
            rc = L.orc_read_binary_page(_ptr(np.ascontiguousarray(page)), length, nv, int(nullable), offset_width, ctypes.byref(bv), _ptr(bits))
            _check(rc, "read_binary_page")
            if nullable:
                valid.append(np.unpackbits(bits, bitorder="little")[:nv].astype(bool))
            pos += length
        offs = np.ctypeslib.as_array(bv.offsets, shape=(bv.n_off,)).copy() if bv.n_off else np.zeros(0, np.int64)
        vals = ctypes.string_at(bv.values, bv.n_val) if bv.n_val else b""
    finally:
        L.orc_binvec_free(ctypes.byref(bv))
    return offs, vals, (np.concatenate(valid) if nullable and valid else None)


def check_utf8(values: bytes, offsets) -> bool:
    """Utf8Array::try_new's check (read/array/binary.rs:305-306), restated from
    arrow2 0.17 `try_check_utf8` (src/array/specification.rs; arrow2 is a
    dependency, Cargo.toml:38, not vendored in the reference): an array of no
    rows passes; else the whole values buffer must be UTF-8 (simdutf8 basic,
    RFC 3629 -- Python's strict decoder accepts exactly that set), and unless
    it is ASCII every offset up to `last` -- the last index >= 1 whose offset
    is below the values length -- must not point at a 0b10xxxxxx byte."""
    offs = [int(x) for x in offsets]
    if len(offs) <= 1:
        return True
    if values.isascii():
        return True
    try:
        values.decode("utf-8", "strict")
    except UnicodeDecodeError:
        return False
    last = next((i for i in range(len(offs) - 1, 0, -1) if offs[i] < len(values)), None)
    if last is None:
        return True
    return all(values[o] & 0xC0 != 0x80 for o in offs[:last + 1])


# ---- nested List<primitive> ---------------------------------------------------
def _list_lib():
    L = lib()
    if not getattr(L, "_list_ready", False):
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.orc_write_list_page.argtypes = [P, P, S, I, P, P, I, I, I, I, ctypes.POINTER(WriteOptions), ctypes.POINTER(_Buf),
                                          ctypes.POINTER(ctypes.c_uint64)]
        L.orc_read_list_page.argtypes = [P, S, S, I, I, I, I, P, P, P, P, ctypes.POINTER(S), ctypes.POINTER(S)]
        L._list_ready = True
    return L


def write_list_column(offsets, list_validity, child, child_validity, list_nullable, item_nullable, page_rows, opts=None):
    """encode_chunk for one List<T> leaf: pages of page_rows top-level rows;
    returns (chunk, [(length, num_levels)], [rows per page])."""
    L = _list_lib()
    opts = opts or WriteOptions.make()
    offsets = np.ascontiguousarray(offsets, np.int64)
    child = np.ascontiguousarray(child)
    rows = len(offsets) - 1
    lvb = None if list_validity is None else np.packbits(np.asarray(list_validity, bool), bitorder="little")
    cvb = None if child_validity is None else np.packbits(np.asarray(child_validity, bool), bitorder="little")
    kind = 1 if child.dtype.kind == "f" else 0
    pages, metas, prow = [], [], []
    step = page_rows or max(rows, 1)
    for r0 in range(0, rows, step):
        m = min(step, rows - r0)
        sub_lv = None
        if lvb is not None:
            sub_lv = np.packbits(np.asarray(list_validity, bool)[r0:r0 + m], bitorder="little")
        buf = _Buf()
        nlev = ctypes.c_uint64()
        rc = L.orc_write_list_page(_ptr(offsets[r0:r0 + m + 1].copy()), _ptr(sub_lv), m, int(list_nullable),
                                   _ptr(child), _ptr(cvb), int(item_nullable), kind, child.itemsize,
                                   int(child.dtype.kind == "i"), ctypes.byref(opts), ctypes.byref(buf), ctypes.byref(nlev))
        pg = _take(buf)
        _check(rc, "write_list_page")
        pages.append(pg)
        metas.append((len(pg), nlev.value))
        prow.append(m)
    return b"".join(pages), metas, prow


def read_list_column(chunk, metas, dtype, list_nullable, item_nullable):
    """batch read of a List<T> leaf: per page create_list, then concatenate
    -> (offsets int64 rows+1, list validity|None, values, leaf validity|None)."""
    L = _list_lib()
    dtype = np.dtype(dtype)
    src = np.frombuffer(chunk, np.uint8)
    offs_all, lv_all, vals_all, leafv_all = [np.zeros(1, np.int64)], [], [], []
    base = 0
    pos = 0
    kind = 1 if dtype.kind == "f" else 0
    for length, nlev in metas:
        page = np.ascontiguousarray(src[pos:pos + length])
        offs = np.zeros(nlev + 1, np.int64)
        lbits = np.zeros(nlev // 8 + 2, np.uint8)
        vals = np.zeros(nlev + 1, dtype)
        fbits = np.zeros(nlev // 8 + 2, np.uint8)
        nr, nleaf = ctypes.c_size_t(), ctypes.c_size_t()
        rc = L.orc_read_list_page(_ptr(page), length, nlev, int(list_nullable), int(item_nullable), kind, dtype.itemsize,
                                  _ptr(offs), _ptr(lbits), _ptr(vals), _ptr(fbits), ctypes.byref(nr), ctypes.byref(nleaf))
        _check(rc, "read_list_page")
        r, v = nr.value, nleaf.value
        offs_all.append(offs[1:r].copy() + base)
        offs_all.append(np.array([v + base], np.int64))
        base += v
        if list_nullable:
            lv_all.append(np.unpackbits(lbits, bitorder="little")[:r].astype(bool))
        vals_all.append(vals[:v])
        if item_nullable:
            leafv_all.append(np.unpackbits(fbits, bitorder="little")[:v].astype(bool))
        pos += length
    offsets = np.concatenate(offs_all)
    return (offsets, np.concatenate(lv_all) if list_nullable else None, np.concatenate(vals_all),
            np.concatenate(leafv_all) if item_nullable else None)


def read_nested_column(chunk, metas, dtype, list_nullable, item_nullable, leaf="fixed", offset_width=4,
                       struct_mask=0, with_counts=False):
    """batch read of a leaf under len(list_nullable) nests (outermost first;
    bit d of struct_mask: nest d is a Struct, else a List / Map): per page
    orc_read_nest_page, then the pages concatenated with each list level's
    offsets moved onto its child's running length ->
    ([offsets per nest | None for structs], [validity per nest | None],
     values, leaf validity | None), and with_counts: a fifth item, the
    entries of every nest and the leaf slots.
    leaf="binary": values = (offsets int64, bytes) of the concatenated per-page
    Utf8 arrays (each page's values[p0:pn], arrow concatenate);
    leaf="bool": values = a bool array."""
    L = _bin_lib()
    if not getattr(L, "_nested_ready", False):
        P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.orc_read_nest_page.argtypes = [P, S, S, I, P, ctypes.c_uint32, I, I, I, P, P, P, P, P, ctypes.POINTER(S)]
        L._nested_ready = True
    struct_mask = int(struct_mask or 0)
    dtype = np.dtype(dtype)
    D = len(list_nullable)
    src = np.frombuffer(chunk, np.uint8)
    kind = {"binary": 2, "bool": 3}.get(leaf, 1 if dtype.kind == "f" else 0)
    width = offset_width if leaf == "binary" else dtype.itemsize
    bin_offs, bin_vals, vbase = [np.zeros(1, np.int64)], [], 0
    offs = [[] for _ in range(D)]
    bits = [[] for _ in range(D)]
    vals, leafv = [], []
    base = [0] * (D + 1)
    pos = 0
    ln = (ctypes.c_int * D)(*[int(x) for x in list_nullable])
    for length, nlev in metas:
        page = np.ascontiguousarray(src[pos:pos + length])
        o = [np.zeros(nlev + 1, np.int64) for _ in range(D)]
        b = [np.zeros(nlev // 8 + 2, np.uint8) for _ in range(D)]
        v = np.zeros(nlev + 1, dtype) if kind < 2 else np.zeros(nlev // 8 + 2, np.uint8)
        fb = np.zeros(nlev // 8 + 2, np.uint8)
        op = (ctypes.c_void_p * D)(*[None if (struct_mask >> d) & 1 else x.ctypes.data for d, x in enumerate(o)])
        bp = (ctypes.c_void_p * D)(*[x.ctypes.data for x in b])
        cnt = (ctypes.c_size_t * (D + 1))()
        rows = ctypes.c_size_t()
        bv = _BinVec()
        vptr = ctypes.addressof(bv) if kind == 2 else _ptr(v)
        try:
            rc = L.orc_read_nest_page(_ptr(page), length, nlev, D, ln, struct_mask, int(item_nullable), kind, width,
                                      op, bp, vptr, _ptr(fb), cnt, ctypes.byref(rows))
            _check(rc, "read_nested_page")
            if kind == 2:
                po = np.ctypeslib.as_array(bv.offsets, shape=(bv.n_off,)).copy() if bv.n_off else np.zeros(1, np.int64)
                pv = ctypes.string_at(bv.values, bv.n_val) if bv.n_val else b""
                bin_offs.append(po[1:] - po[0] + vbase)
                bin_vals.append(pv[po[0]:po[-1]])
                vbase += int(po[-1] - po[0])
        finally:
            L.orc_binvec_free(ctypes.byref(bv))
        for d in range(D):
            offs[d].append(o[d][:cnt[d]] + base[d + 1])
            if list_nullable[d]:
                bits[d].append(np.unpackbits(b[d], bitorder="little")[:cnt[d]].astype(bool))
        if kind < 2:
            vals.append(v[:cnt[D]])
        elif kind == 3:
            vals.append(np.unpackbits(v, bitorder="little")[:cnt[D]].astype(bool))
        if item_nullable:
            leafv.append(np.unpackbits(fb, bitorder="little")[:cnt[D]].astype(bool))
        for d in range(D + 1):
            base[d] += cnt[d]
        pos += length
    out_offs = [None if (struct_mask >> d) & 1 else np.concatenate(offs[d] + [np.array([base[d + 1]], np.int64)])
                for d in range(D)]
    out_bits = [np.concatenate(bits[d]) if list_nullable[d] else None for d in range(D)]
    values = (np.concatenate(bin_offs), b"".join(bin_vals)) if kind == 2 else np.concatenate(vals)
    if with_counts:
        return out_offs, out_bits, values, (np.concatenate(leafv) if item_nullable else None), list(base)
    return out_offs, out_bits, values, (np.concatenate(leafv) if item_nullable else None)


# ---- boolean pages (compression/boolean/*.rs, read/array/boolean.rs) ---------
def _pack(b) -> np.ndarray:
    return np.packbits(np.asarray(b, bool), bitorder="little")


def write_bool_page(values, validity=None, nullable=False, opts: WriteOptions | None = None, offset: int = 0,
                    n: int | None = None) -> bytes:
    """One flat boolean page.  values = the whole column's bools; the page is
    rows [offset, offset + n) (array.slice), so the Basic codec sees the
    parent bitmap's bytes when offset % 8 == 0 (boolean/mod.rs:35-46).
    validity (page-relative) has n entries."""
    vals = np.asarray(values, bool)
    n = len(vals) - offset if n is None else n
    bits = _pack(vals)
    if len(bits) == 0:
        bits = np.zeros(1, np.uint8)
    vb = None if validity is None else _pack(validity)
    buf = _Buf()
    rc = lib().orc_write_bool_page(_ptr(bits), offset, _ptr(vb), n, int(nullable), ctypes.byref(opts or WriteOptions.make()),
                                   ctypes.byref(buf))
    data = _take(buf)
    _check(rc, "write_bool_page")
    return data


def read_bool_page(page: bytes, n: int, nullable=False):
    src = _bytes_arr(page)
    vb = np.zeros((n + 7) // 8 + 1, np.uint8)
    mb = np.zeros((n + 7) // 8 + 1, np.uint8)
    _check(lib().orc_read_bool_page(_ptr(src), len(page), n, int(nullable), _ptr(vb), _ptr(mb)), "read_bool_page")
    vals = np.unpackbits(vb, bitorder="little")[:n].astype(bool)
    return vals, (np.unpackbits(mb, bitorder="little")[:n].astype(bool) if nullable else None)


def read_bool_column(chunk: bytes, metas, nullable=False):
    """read_boolean (read/array/boolean.rs:191-219) -> (values bits, validity bits|None) as bool arrays."""
    n = sum(int(m[1]) for m in metas)
    flat = np.asarray([int(x) for m in metas for x in m], np.uint64)
    src = _bytes_arr(chunk)
    vb = np.zeros((n + 7) // 8 + 1, np.uint8)
    mb = np.zeros((n + 7) // 8 + 1, np.uint8)
    _check(lib().orc_read_bool_column(_ptr(src), len(chunk), _ptr(flat), len(metas), int(nullable), _ptr(vb), _ptr(mb)),
           "read_bool_column")
    vals = np.unpackbits(vb, bitorder="little")[:n].astype(bool)
    return vals, (np.unpackbits(mb, bitorder="little")[:n].astype(bool) if nullable else None)


# ---- multi-threaded CPU baseline (sb_cpu_mt.c) ------------------------------
def _mt_lib():
    L = lib()
    if not getattr(L, "_mt_ready", False):
        P, S, I, U64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        L.orc_mt_read_column.argtypes = [P, P, S, I, I, I, P, P, I]
        L.orc_mt_read_binary_column.argtypes = [P, P, S, I, I, P, P, U64, P, I, ctypes.POINTER(U64)]
        L.orc_mt_read_list_column.argtypes = [P, P, S, I, I, I, I, P, P, P, P, I, ctypes.POINTER(U64),
                                              ctypes.POINTER(U64)]
        L.orc_mt_read_bool_column.argtypes = [P, P, S, I, P, P, I]
        L._mt_ready = True
    return L


def _metas(metas):
    return np.asarray([(int(l), int(nv)) for l, nv in metas], dtype=np.uint64).reshape(-1)


def mt_read_column(chunk, metas, dtype, nullable, threads, out=None):
    """read_integer / read_double with the pages sharded over `threads`
    workers -> (values, validity bytes|None).  `out` = preallocated buffers."""
    dtype = np.dtype(dtype)
    n = sum(int(nv) for _, nv in metas)
    src = chunk if isinstance(chunk, np.ndarray) else np.frombuffer(chunk, np.uint8)
    vals, bits = out if out is not None else (np.empty(max(n, 1), dtype), np.zeros(n // 8 + 2, np.uint8))
    m = _metas(metas)
    _check(_mt_lib().orc_mt_read_column(_ptr(src), _ptr(m), len(metas), int(dtype.kind == "f"), dtype.itemsize,
                                        int(nullable), _ptr(vals), _ptr(bits), threads), "mt_read_column")
    return vals, (bits if nullable else None)


def mt_read_binary_column(chunk, metas, nullable, ow, threads, values_cap, out=None):
    """read_binary with pages sharded over workers -> (offsets, values, bits|None, values_len)."""
    n = sum(int(nv) for _, nv in metas)
    src = chunk if isinstance(chunk, np.ndarray) else np.frombuffer(chunk, np.uint8)
    offs, vals, bits = out if out is not None else (np.empty(n + 1, np.int64 if ow == 8 else np.int32),
                                                    np.empty(max(values_cap, 1), np.uint8),
                                                    np.zeros(n // 8 + 2, np.uint8))
    vl = ctypes.c_uint64()
    m = _metas(metas)
    _check(_mt_lib().orc_mt_read_binary_column(_ptr(src), _ptr(m), len(metas), int(nullable), ow, _ptr(offs),
                                               _ptr(vals), len(vals), _ptr(bits), threads, ctypes.byref(vl)),
           "mt_read_binary_column")
    return offs, vals, (bits if nullable else None), vl.value


def mt_read_list_column(chunk, metas, dtype, list_nullable, item_nullable, threads, out=None):
    """List<T> batch read with pages sharded over workers ->
    (offsets int64, list bits|None, values, leaf bits|None, rows, leaves)."""
    dtype = np.dtype(dtype)
    lev = sum(int(nv) for _, nv in metas)
    src = chunk if isinstance(chunk, np.ndarray) else np.frombuffer(chunk, np.uint8)
    offs, lb, vals, fb = out if out is not None else (np.empty(lev + 2, np.int64), np.zeros(lev // 8 + 2, np.uint8),
                                                      np.empty(lev + 1, dtype), np.zeros(lev // 8 + 2, np.uint8))
    r, v = ctypes.c_uint64(), ctypes.c_uint64()
    m = _metas(metas)
    _check(_mt_lib().orc_mt_read_list_column(_ptr(src), _ptr(m), len(metas), int(list_nullable), int(item_nullable),
                                             int(dtype.kind == "f"), dtype.itemsize, _ptr(offs), _ptr(lb), _ptr(vals),
                                             _ptr(fb), threads, ctypes.byref(r), ctypes.byref(v)),
           "mt_read_list_column")
    return offs, (lb if list_nullable else None), vals, (fb if item_nullable else None), r.value, v.value


def mt_read_bool_column(chunk, metas, nullable, threads, out=None):
    n = sum(int(nv) for _, nv in metas)
    src = chunk if isinstance(chunk, np.ndarray) else np.frombuffer(chunk, np.uint8)
    vb, mb = out if out is not None else (np.zeros(n // 8 + 2, np.uint8), np.zeros(n // 8 + 2, np.uint8))
    m = _metas(metas)
    _check(_mt_lib().orc_mt_read_bool_column(_ptr(src), _ptr(m), len(metas), int(nullable), _ptr(vb), _ptr(mb),
                                             threads), "mt_read_bool_column")
    return vb, (mb if nullable else None)
