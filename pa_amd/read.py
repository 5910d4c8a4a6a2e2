"""Read side of the strawboat engine, mirroring the reference's API names.

Reference (b41sh/pa @ 2025-01-17):
  PageMeta / ColumnMeta          src/lib.rs:40-80
  read_meta                      src/read/reader.rs:168-178
  NativeReader                   src/read/reader.rs:51-146
  column_iter_to_arrays          src/read/deserialize.rs:237-253 (one array per page)
  batch_read_array               src/read/batch_read.rs:190-209 (one array per column)

Device memory and streams come from torch (ROCm); every decode is a launch
of the HIP kernels in libstrawboat_gpu.so through its C ABI.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N

_PHYS = {
    np.dtype(np.int8): N.INT8, np.dtype(np.int16): N.INT16, np.dtype(np.int32): N.INT32,
    np.dtype(np.int64): N.INT64, np.dtype(np.uint8): N.UINT8, np.dtype(np.uint16): N.UINT16,
    np.dtype(np.uint32): N.UINT32, np.dtype(np.uint64): N.UINT64, np.dtype(np.float32): N.FLOAT32,
    np.dtype(np.float64): N.FLOAT64, np.dtype(np.bool_): N.BOOLEAN,
}


def physical_type(dtype) -> int:
    dt = np.dtype(dtype)
    if dt not in _PHYS:
        raise N.StrawboatError(N.E_NYI, f"physical type {dt} not supported")
    return _PHYS[dt]


@dataclass(frozen=True)
class PageMeta:
    """src/lib.rs:75-80: compressed page length and its num_values."""

    length: int
    num_values: int


@dataclass
class ColumnMeta:
    """src/lib.rs:40-70."""

    offset: int
    pages: List[PageMeta] = field(default_factory=list)

    def slice(self, start: int, end: int) -> "ColumnMeta":
        assert start < len(self.pages) and end <= len(self.pages)
        off = self.offset + sum(p.length for p in self.pages[:start])
        return ColumnMeta(off, list(self.pages[start:end]))

    def skip_one_page(self) -> "ColumnMeta":
        return self.slice(1, len(self.pages))

    def total_len(self) -> int:
        return sum(p.length for p in self.pages)


def read_meta(file_bytes: bytes) -> List[ColumnMeta]:
    """read_meta (reader.rs:168-178) through sb_read_meta."""
    L = N.lib()
    buf = (ctypes.c_uint8 * len(file_bytes)).from_buffer_copy(file_bytes)
    nc, npg = ctypes.c_uint64(), ctypes.c_uint64()
    st = L.sb_read_meta(buf, len(file_bytes), None, None, 0, None, 0, ctypes.byref(nc), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "read_meta")
    offs = (ctypes.c_uint64 * max(1, nc.value))()
    starts = (ctypes.c_uint64 * max(1, nc.value))()
    pages = (N.PageMetaC * max(1, npg.value))()
    st = L.sb_read_meta(buf, len(file_bytes), offs, starts, nc.value, pages, npg.value, ctypes.byref(nc), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "read_meta")
    metas = []
    for c in range(nc.value):
        end = starts[c + 1] if c + 1 < nc.value else npg.value
        metas.append(ColumnMeta(offs[c], [PageMeta(pages[i].length, pages[i].num_values) for i in range(starts[c], end)]))
    return metas


class NativeReader:
    """Host page iterator (reader.rs:51-146): yields (num_values, page bytes)."""

    def __init__(self, data: bytes, page_metas: Sequence[PageMeta], offset: int = 0):
        self._data = memoryview(data)
        self._metas = list(page_metas)
        self._pos = offset
        self.current_page = 0

    def has_next(self) -> bool:
        return self.current_page < len(self._metas)

    def __iter__(self):
        return self

    def __next__(self) -> Tuple[int, bytes]:
        if not self.has_next():
            raise StopIteration
        m = self._metas[self.current_page]
        b = bytes(self._data[self._pos:self._pos + m.length])
        if len(b) != m.length:
            raise N.StrawboatError(N.E_IO, "short page read")
        self._pos += m.length
        self.current_page += 1
        return m.num_values, b

    def skip_page(self):
        if self.has_next():
            self._pos += self._metas[self.current_page].length
            self.current_page += 1


class Context:
    """One sb_ctx = one device + one HIP stream (torch's current stream)."""

    def __init__(self, device: int = 0):
        import torch

        self.device = device
        self._torch = torch
        h = ctypes.c_void_p()
        st = N.lib().sb_ctx_create(device, ctypes.byref(h))
        if st:
            raise N.StrawboatError(st, f"sb_ctx_create(device={device}) failed: no usable GPU")
        self._h = h
        self._own = N.lib().sb_ctx_stream(h)  # the context's own HIP stream (non-blocking)
        with torch.cuda.device(device):
            self.use_stream(torch.cuda.current_stream(device))

    def use_stream(self, stream):
        N.lib().sb_ctx_set_stream(self._h, ctypes.c_void_p(stream.cuda_stream))

    def use_own_stream(self):
        """Launch on the context's own HIP stream; returns it as a torch
        ExternalStream (for wait_stream / stream contexts).  Contexts created
        one after another get their own streams on distinct hardware queues
        (the runtime spreads new streams over its queues), where torch's
        pooled side streams may share one -- independent columns then
        really run side by side."""
        st = self._torch.cuda.ExternalStream(self._own, device=self.device)
        self.use_stream(st)
        return st

    def error(self) -> str:
        return N.lib().sb_last_error(self._h).decode()

    def close(self):
        if getattr(self, "_h", None):
            N.lib().sb_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device: Optional[int] = None) -> Context:
    """The shared context of `device` (default: torch's current device)."""
    if device is None:
        import torch

        device = torch.cuda.current_device()
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def resolve_context(ctx: Optional[Context], data=None) -> Context:
    """ctx as given, else the default context of the device `data` (a tensor)
    lives on, else of torch's current device.  A device tensor on another
    device than ctx is an argument error: the kernels would read it through
    a peer mapping and write their outputs on the wrong GPU."""
    dev = data.device.index if getattr(data, "is_cuda", False) else None
    if ctx is None:
        return default_context(dev)
    if dev is not None and dev != ctx.device:
        raise N.StrawboatError(N.E_ARG, f"tensor on cuda:{dev} but context on cuda:{ctx.device}")
    return ctx


def _as_device_bytes(chunk, device):
    import torch

    if isinstance(chunk, torch.Tensor):
        if chunk.dtype != torch.uint8 or not chunk.is_cuda:
            raise N.StrawboatError(N.E_ARG, "column chunk must be a uint8 device tensor or host bytes")
        if chunk.device.index != device:
            raise N.StrawboatError(N.E_ARG, f"chunk on cuda:{chunk.device.index} but context on cuda:{device}")
        return chunk.contiguous()
    arr = np.frombuffer(bytes(chunk), dtype=np.uint8)
    return torch.from_numpy(arr.copy()).to(f"cuda:{device}")


class ColumnDecoder:
    """A planned column chunk: device page table built once, decoded many times.

    decode() is the batch_read_array path for one flat primitive leaf
    (batch_read.rs:27-60 -> read_integer / read_double)."""

    def __init__(self, chunk, page_metas: Sequence[PageMeta], dtype, nullable: bool, ctx: Optional[Context] = None,
                 timing: bool = False):
        import torch

        self.ctx = resolve_context(ctx, chunk)
        self.dtype = np.dtype(dtype)
        self.nullable = bool(nullable)
        self.chunk = _as_device_bytes(chunk, self.ctx.device)
        self.metas = list(page_metas)
        metas = (N.PageMetaC * max(1, len(self.metas)))(*[N.PageMetaC(m.length, m.num_values) for m in self.metas])
        desc = N.ColumnDescC(physical_type(self.dtype), int(self.nullable))
        h = ctypes.c_void_p()
        st = N.lib().sb_plan_column(self.ctx._h, ctypes.byref(desc), ctypes.c_void_p(self.chunk.data_ptr()),
                                    self.chunk.numel(), metas, len(self.metas), ctypes.byref(h))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        self._h = h
        if timing:
            N.lib().sb_plan_enable_timing(h, 1)
        self.num_rows = int(N.lib().sb_plan_num_rows(h))
        self._torch = torch

    @classmethod
    def for_shard(cls, chunk, page_metas, shard, dtype, nullable: bool, ctx=None, timing: bool = False):
        """The decoder of one rank's page range (pa_amd.shard_pages): only the
        shard's bytes are planned and decoded; rows start at shard.row_offset
        of the whole column."""
        from .shard import shard_slice

        part, metas = shard_slice(chunk, page_metas, shard)
        dec = cls(part, metas, dtype, nullable, ctx, timing)
        dec.shard = shard
        return dec

    def alloc_outputs(self):
        torch = self._torch
        dev = f"cuda:{self.ctx.device}"
        if self.dtype == np.bool_:  # read_boolean: the values are a bitmap, laid out like the validity
            nwords = (self.num_rows + 31) // 32
            values = torch.zeros(max(nwords, 1) * 4, dtype=torch.uint8, device=dev)
        else:
            tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[self.dtype.itemsize]
            values = torch.empty(max(self.num_rows, 1), dtype=tdt, device=dev)
        validity = None
        if self.nullable:
            nwords = (self.num_rows + 31) // 32
            validity = torch.zeros(max(nwords, 1) * 4, dtype=torch.uint8, device=dev)
        return values, validity

    def decode_async(self, values=None, validity=None):
        if values is None:
            values, validity = self.alloc_outputs()
        out = N.PrimitiveOutC(values.data_ptr(), validity.data_ptr() if validity is not None else None)
        st = N.lib().sb_decode_planned(self.ctx._h, self._h, ctypes.byref(out))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        return values, validity

    def check(self):
        bad = ctypes.c_int64(-1)
        st = N.lib().sb_plan_status(self.ctx._h, self._h, ctypes.byref(bad))
        if st:
            raise N.StrawboatError(st, self.ctx.error())

    def decode(self, values=None, validity=None):
        v, m = self.decode_async(values, validity)
        self.check()
        return v, m

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        st = N.lib().sb_plan_last_kernel_ms(self.ctx._h, self._h, ctypes.byref(ms))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        return ms.value

    def close(self):
        if getattr(self, "_h", None):
            N.lib().sb_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def batch_read_array(chunk, page_metas: Sequence[PageMeta], dtype, nullable: bool, ctx: Optional[Context] = None):
    """batch_read_array (batch_read.rs:190-209) for a flat primitive leaf:
    returns (values, validity_bitmap|None) as device tensors (values typed by
    width; view as the logical dtype with values.view(...); Boolean values
    are a bitmap like the validity)."""
    dec = ColumnDecoder(chunk, page_metas, dtype, nullable, ctx)
    try:
        return dec.decode()
    finally:
        dec.close()


def column_iter_to_arrays(chunk, page_metas: Sequence[PageMeta], dtype, nullable: bool,
                          ctx: Optional[Context] = None) -> Iterator[Tuple[object, Optional[object]]]:
    """column_iter_to_arrays (deserialize.rs:237-253): one (values, validity)
    per page.  All pages decode in one batched launch; each yielded array is
    a slice of it (validity as a bool tensor)."""
    values, bitmap = batch_read_array(chunk, page_metas, dtype, nullable, ctx)
    valid_bool = unpack_bitmap(bitmap, sum(m.num_values for m in page_metas)) if nullable else None
    row = 0
    for m in page_metas:
        n = m.num_values
        yield values[row:row + n], (valid_bool[row:row + n] if valid_bool is not None else None)
        row += n


def unpack_bitmap(bitmap, n: int):
    """LSB-first Arrow bitmap -> bool tensor of n entries (on device)."""
    torch = __import__("torch")
    bits = torch.arange(8, device=bitmap.device, dtype=torch.uint8)
    b = (bitmap[: (n + 7) // 8].unsqueeze(1) >> bits) & 1
    return b.reshape(-1)[:n].bool()


def read_validity(page, length: int, out=None, bit_offset: int = 0, ctx: Optional[Context] = None):
    """read_validity (read/read_basic.rs:36-63) of one flat nullable page on
    the GPU (sb_decode_page_validity): page = its bytes (host bytes or a
    device uint8 tensor).  Writes `length` bits at bit_offset of out (a device
    int32 bitmap tensor, allocated when None) and returns (out, bytes of the
    prefix: the values stream starts there)."""
    import torch

    ctx = resolve_context(ctx, page)
    d = _as_device_bytes(page, ctx.device)
    if out is None:
        out = torch.zeros(max((bit_offset + length + 31) // 32, 1), dtype=torch.int32, device=f"cuda:{ctx.device}")
    used = ctypes.c_uint64()
    st = N.lib().sb_decode_page_validity(ctx._h, ctypes.c_void_p(d.data_ptr()), d.numel(), length,
                                         ctypes.c_void_p(out.data_ptr()), bit_offset, ctypes.byref(used))
    if st:
        raise N.StrawboatError(st, ctx.error())
    return out, used.value


def read_levels(page, num_levels: int, max_rep_level: int, max_def_level: int, ctx: Optional[Context] = None):
    """The rep / def level streams of one nested page (read_validity_nested,
    read/read_basic.rs:65-86) on the GPU (sb_decode_page_levels) -> (rep,
    def device int16 tensors of num_levels levels, the page's row count, the
    header + level bytes)."""
    import torch

    ctx = resolve_context(ctx, page)
    d = _as_device_bytes(page, ctx.device)
    dev = f"cuda:{ctx.device}"
    rep = torch.empty(max(num_levels, 1), dtype=torch.int16, device=dev)
    dfl = torch.empty(max(num_levels, 1), dtype=torch.int16, device=dev)
    rows, used = ctypes.c_uint32(), ctypes.c_uint64()
    st = N.lib().sb_decode_page_levels(ctx._h, ctypes.c_void_p(d.data_ptr()), d.numel(), num_levels, max_rep_level,
                                       max_def_level, ctypes.c_void_p(rep.data_ptr()), ctypes.c_void_p(dfl.data_ptr()),
                                       ctypes.byref(rows), ctypes.byref(used))
    if st:
        raise N.StrawboatError(st, ctx.error())
    return rep[:num_levels], dfl[:num_levels], rows.value, used.value
