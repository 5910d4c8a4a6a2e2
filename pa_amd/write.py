"""Write side, mirroring the reference's NativeWriter / WriteOptions.

Reference (b41sh/pa @ 2025-01-17):
  WriteOptions                  src/write/common.rs:37-45
  NativeWriter::{new, start, write, finish}   src/write/writer.rs:42-167
  encode_chunk (paging)         src/write/common.rs:49-119

Encoding runs in the engine's host encoder (libstrawboat_gpu.so,
sb_encode_column); pages are encoded in parallel on the host's cores.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .read import ColumnMeta, PageMeta, physical_type

# CommonCompression / Compression codec ids (compression/mod.rs:64-82)
NONE, LZ4, ZSTD, SNAPPY = 0, 1, 2, 3
RLE, DICT, ONE_VALUE, FREQ, BITPACKING, DELTA_BITPACKING, PATAS = 10, 11, 12, 13, 14, 15, 16

ARROW_MAGIC = b"ARROW2"


@dataclass
class WriteOptions:
    """write::WriteOptions (common.rs:37-45).  forced_codec mirrors the
    debug-build STRAWBOAT_*_COMPRESSION switches (util/env.rs); seed drives
    the deterministic trial-window sampler."""

    default_compression: int = NONE
    default_compress_ratio: Optional[float] = None
    max_page_size: Optional[int] = None
    forbidden_compressions: Sequence[int] = field(default_factory=tuple)
    forced_codec: int = -1
    seed: int = 42

    def c(self) -> N.WriteOptionsC:
        m = 0
        for c in self.forbidden_compressions:
            m |= 1 << c
        r = self.default_compress_ratio
        return N.WriteOptionsC(self.default_compression, r is not None, float(r or 0.0), m, self.forced_codec, self.seed)


def _take(ptr, n) -> bytes:
    b = ctypes.string_at(ptr, n) if n else b""
    N.lib().sb_free(ptr)
    return b


def encode_column(values: np.ndarray, validity=None, nullable: bool = False,
                  options: Optional[WriteOptions] = None, n_threads: int = 0) -> Tuple[bytes, List[PageMeta]]:
    """encode_chunk for one flat leaf -> (column chunk bytes, page metas)."""
    options = options or WriteOptions()
    values = np.ascontiguousarray(values)
    n = len(values)
    phys = physical_type(values.dtype)
    if phys == N.BOOLEAN:  # compress_boolean takes the column's bitmap; pages slice it
        values = np.packbits(values, bitorder="little")
        if len(values) == 0:
            values = np.zeros(1, np.uint8)
    vb = None
    if validity is not None:
        vb = np.packbits(np.asarray(validity, bool), bitorder="little")
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    metas = ctypes.POINTER(N.PageMetaC)()
    npg = ctypes.c_uint64()
    opts = options.c()
    st = N.lib().sb_encode_column(
        phys, values.ctypes.data_as(ctypes.c_void_p),
        None if vb is None else vb.ctypes.data_as(ctypes.c_void_p), n, int(nullable),
        ctypes.byref(opts), options.max_page_size or 0, n_threads, ctypes.byref(out), ctypes.byref(olen),
        ctypes.byref(metas), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "encode_column")
    pm = [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]
    N.lib().sb_free(metas)
    return _take(out, olen.value), pm


def encode_column_device(values, validity=None, nullable: bool = False, options: Optional[WriteOptions] = None,
                         ctx=None):
    """encode_chunk on the GPU (sb_encode_column_device): values is a device
    tensor of a fixed-width type or bool, validity an optional device bool
    tensor.  Every option of the reference's writer runs on the device --
    the adaptive cascade with the seeded sampler, forced codecs, Basic None /
    LZ4 / Snappy -- except a Zstd default codec (NotYetImplemented).
    Returns (device uint8 tensor of the column chunk, page metas),
    byte-identical to encode_column with the same options."""
    import torch

    from .read import resolve_context

    options = options or WriteOptions()
    ctx = resolve_context(ctx, values)
    values = values.contiguous()
    n = values.numel()

    def pack(bits):  # bool device tensor -> LSB-first bitmap bytes (at least one byte)
        pad = (-n) % 8
        if pad:
            bits = torch.cat([bits, torch.zeros(pad, dtype=torch.bool, device=bits.device)])
        w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=bits.device)
        if not n:
            return torch.zeros(1, dtype=torch.uint8, device=bits.device)
        return (bits.view(-1, 8).to(torch.uint8) * w).sum(1, dtype=torch.uint8)

    if values.dtype == torch.bool:  # compress_boolean takes the column's bitmap; pages slice it
        phys = N.BOOLEAN
        values = pack(values.reshape(-1))
    else:
        tdt = {torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32, torch.int64: np.int64,
               torch.uint8: np.uint8, torch.uint16: np.uint16, torch.uint32: np.uint32, torch.uint64: np.uint64,
               torch.float32: np.float32, torch.float64: np.float64}[values.dtype]
        phys = physical_type(np.dtype(tdt))
    vb = None
    if nullable:
        # a missing bitmap is all-valid (write_def_levels' (is_optional, None) case), as in encode_column
        vb = pack(validity.to(device=values.device, dtype=torch.bool).reshape(-1) if validity is not None
                  else torch.ones(n, dtype=torch.bool, device=values.device))
    # page_size = max_page_size.unwrap_or(len).min(len) (write/common.rs:54-58)
    P = min(options.max_page_size or n, n)
    cap = N.lib().sb_encode_device_bound(phys, n, int(nullable), P)
    out = torch.empty(max(cap, 16), dtype=torch.uint8, device=values.device)
    npages = (n + P - 1) // P if n else 0
    metas = (N.PageMetaC * max(npages, 1))()
    olen, npg = ctypes.c_uint64(), ctypes.c_uint64()
    opts = options.c()
    st = N.lib().sb_encode_column_device(
        ctx._h, phys, ctypes.c_void_p(values.data_ptr()), None if vb is None else ctypes.c_void_p(vb.data_ptr()), n,
        int(nullable), ctypes.byref(opts), P, ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(olen),
        metas, max(npages, 1), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "encode_column_device: " + ctx.error())
    return out[: olen.value], [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]


@dataclass
class DeviceColumn:
    """One leaf of a chunk for encode_table_device: device tensors of the
    values (and, for Binary / Utf8 leaves, int64 offsets), optional validity."""

    values: object
    validity: object = None
    nullable: bool = False
    options: Optional[WriteOptions] = None
    offsets: object = None      # Binary / Utf8: n + 1 absolute positions into values
    physical_type: int = 0      # Binary / Utf8: pa_amd.UTF8 ...; 0 = from the values' dtype


_table_ctx = {}


def _table_contexts(device: int, n: int):
    """n contexts of this device, each on its own torch side stream (cached:
    their grow-only scratch is reused by the next table)."""
    import torch

    from .read import Context

    key = (device, n)
    if key not in _table_ctx:
        ctxs = []
        for _ in range(n):  # (own streams: on distinct hardware queues, Context.use_own_stream)
            c = Context(device)
            ctxs.append((c, c.use_own_stream()))
        _table_ctx[key] = ctxs
    return _table_ctx[key]


def encode_table_device(columns: Sequence[DeviceColumn], n_streams: int = 4, device: Optional[int] = None):
    """encode_chunk for every leaf of a chunk on the GPU (NativeWriter::write,
    write/writer.rs:113-143, encodes the chunk's columns one after another;
    they are independent, so here up to n_streams of them are in flight at
    once, each through its own context and HIP stream).  A page's Basic LZ4
    stream is one serial parse (latency-bound on one wave), so columns made
    of such pages go first and overlap the rest.  Returns [(device uint8
    chunk, page metas)] in column order, each byte-identical to the host
    writer's (encode_column / encode_binary_column)."""
    import threading

    import torch

    from .binary import encode_binary_column_device

    cols = list(columns)
    if not cols:
        return []
    dev = cols[0].values.device.index if device is None else device
    ctxs = _table_contexts(dev, max(1, n_streams))
    cur = torch.cuda.current_stream(dev)
    for _, st in ctxs:
        st.wait_stream(cur)  # the inputs were produced on the caller's stream

    def cost(i):
        o = cols[i].options or WriteOptions()
        serial = o.default_compress_ratio is None and o.default_compression in (LZ4, SNAPPY)
        return (not serial, -cols[i].values.numel() * cols[i].values.element_size())

    order = sorted(range(len(cols)), key=cost)
    out = [None] * len(cols)
    lock = threading.Lock()
    errors = []

    def worker(k):
        ctx, st = ctxs[k]
        try:
            with torch.cuda.device(dev), torch.cuda.stream(st):
                while True:
                    with lock:
                        if not order or errors:
                            return
                        i = order.pop(0)
                    c = cols[i]
                    if c.offsets is not None:
                        out[i] = encode_binary_column_device(c.values, c.offsets, c.validity, c.nullable, c.options,
                                                             c.physical_type or 13, ctx=ctx)
                    else:
                        out[i] = encode_column_device(c.values, c.validity, c.nullable, c.options, ctx=ctx)
        except Exception as e:  # noqa: BLE001 -- re-raised below, in the caller's thread
            with lock:
                errors.append(e)

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(len(ctxs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    for _, st in ctxs:
        cur.wait_stream(st)
    return out


def encode_page(values: np.ndarray, validity=None, nullable: bool = False,
                options: Optional[WriteOptions] = None, seed: Optional[int] = None) -> bytes:
    options = options or WriteOptions()
    values = np.ascontiguousarray(values)
    vb = None if validity is None else np.packbits(np.asarray(validity, bool), bitorder="little")
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    opts = options.c()
    st = N.lib().sb_encode_page(physical_type(values.dtype), values.ctypes.data_as(ctypes.c_void_p),
                                None if vb is None else vb.ctypes.data_as(ctypes.c_void_p), len(values), int(nullable),
                                ctypes.byref(opts), options.seed if seed is None else seed, ctypes.byref(out),
                                ctypes.byref(olen))
    if st:
        raise N.StrawboatError(st, "encode_page")
    return _take(out, olen.value)


def page_seed(seed: int, page: int) -> int:
    return N.lib().sb_page_seed(seed, page)


class NativeWriter:
    """NativeWriter (writer.rs:42-167) over an in-memory buffer: start() ->
    write(columns) once -> finish(); flat, Binary / Utf8 and nested fields."""

    def __init__(self, options: Optional[WriteOptions] = None, schema_bytes: bytes = b""):
        self.options = options or WriteOptions()
        self.schema_bytes = schema_bytes
        self.buf = bytearray()
        self.metas: List[ColumnMeta] = []
        self.state = "none"

    def start(self):
        if self.state != "none":
            raise N.StrawboatError(N.E_OUT_OF_SPEC, "The strawboat file can only be started once")
        self.buf += ARROW_MAGIC + b"\x00\x00"
        self.state = "started"

    def write(self, columns):
        """columns: one entry per field of the chunk, equal lengths -- a flat
        field as (values, validity|None, nullable), a Binary / Utf8 field as
        (BinaryColumn-like (offsets, bytes) values, validity|None, nullable,
        physical type), a nested field as (pa_amd.Field, pa_amd.HostArray):
        encode_chunk writes every leaf of it, to_leaves order
        (write/common.rs:60-115)."""
        from .nested import Field, encode_field

        if self.state == "written":
            raise N.StrawboatError(N.E_OUT_OF_SPEC, "The strawboat file can only accept one RowGroup in a single file")
        if self.state != "started":
            raise N.StrawboatError(N.E_OUT_OF_SPEC, "The strawboat file must be started before it can be written to")
        for col in columns:
            if isinstance(col[0], Field):
                leaves = encode_field(col[0], col[1], self.options)
            elif len(col) == 4:
                from .binary import encode_binary_column

                (offs, data), validity, nullable, phys = col
                leaves = [encode_binary_column(data, offs, validity, nullable, self.options, phys)]
            else:
                values, validity, nullable = col
                leaves = [encode_column(values, validity, nullable, self.options)]
            for chunk, pages in leaves:
                self.metas.append(ColumnMeta(len(self.buf), pages))
                self.buf += chunk
        self.state = "written"

    def finish(self) -> bytes:
        if self.state != "written":
            raise N.StrawboatError(N.E_OUT_OF_SPEC, "The strawboat file must be written before it can be finished")
        self.buf += footer_bytes(self.metas, self.schema_bytes)
        self.state = "finished"
        return bytes(self.buf)

    def total_size(self) -> int:
        return len(self.buf)


def footer_bytes(metas: Sequence[ColumnMeta], schema_bytes: bytes = b"") -> bytes:
    """The footer NativeWriter::finish writes (writer.rs:128-167): schema,
    column metas, schema size, meta size, EOS."""
    offs = (ctypes.c_uint64 * max(1, len(metas)))(*[m.offset for m in metas])
    nps = (ctypes.c_uint64 * max(1, len(metas)))(*[len(m.pages) for m in metas])
    allp = [p for m in metas for p in m.pages]
    pages = (N.PageMetaC * max(1, len(allp)))(*[N.PageMetaC(p.length, p.num_values) for p in allp])
    sch = (ctypes.c_uint8 * max(1, len(schema_bytes))).from_buffer_copy(schema_bytes or b"\x00")
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    st = N.lib().sb_write_footer(sch, len(schema_bytes), offs, nps, len(metas), pages, ctypes.byref(out),
                                 ctypes.byref(olen))
    if st:
        raise N.StrawboatError(st, "footer")
    return _take(out, olen.value)


def assemble_file(columns: Sequence[Tuple[bytes, Sequence[PageMeta]]], schema_bytes: bytes = b"") -> bytes:
    """A whole file from encoded column chunks (any leaf kind: flat,
    binary, list), in leaf order: header, chunks back to back, footer."""
    buf = bytearray(ARROW_MAGIC + b"\x00\x00")
    metas = []
    for chunk, pages in columns:
        metas.append(ColumnMeta(len(buf), list(pages)))
        buf += chunk
    buf += footer_bytes(metas, schema_bytes)
    return bytes(buf)
