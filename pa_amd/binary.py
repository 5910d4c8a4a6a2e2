"""Binary / Utf8 columns (reference: compression/binary/mod.rs, read/array/binary.rs).

encode_binary_column  -> sb_encode_binary_column  (encode_chunk for one leaf)
BinaryColumnDecoder   -> sb_plan_column (+ device sizing pass) + sb_decode_binary_planned
batch_read_binary     -> read_binary (read/array/binary.rs:223-265): (offsets, values, validity)
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .read import Context, PageMeta, resolve_context, _as_device_bytes

BINARY, LARGE_BINARY, UTF8, LARGE_UTF8 = 11, 12, 13, 14


def _ow(phys: int) -> int:
    return 8 if phys in (LARGE_BINARY, LARGE_UTF8) else 4


def strings_to_arrow(strings: Sequence[bytes]) -> Tuple[bytes, np.ndarray]:
    offs = np.zeros(len(strings) + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in strings])
    return b"".join(strings), offs


def _lib():
    L = N.lib()
    if not getattr(L, "_bin_ready", False):
        P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
        PU8 = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))
        L.sb_encode_binary_column.argtypes = [I32, P, U64, P, P, U64, I32, ctypes.POINTER(N.WriteOptionsC), U64, I32,
                                              PU8, ctypes.POINTER(U64), ctypes.POINTER(ctypes.POINTER(N.PageMetaC)),
                                              ctypes.POINTER(U64)]
        L.sb_encode_binary_column.restype = I32
        L.sb_plan_values_bytes.argtypes = [P]
        L.sb_plan_values_bytes.restype = U64
        L.sb_decode_binary_planned.argtypes = [P, P, ctypes.POINTER(BinaryOutC)]
        L.sb_decode_binary_planned.restype = I32
        L.sb_encode_binary_device_bound.argtypes = [I32, U64, U64, I32, U64]
        L.sb_encode_binary_device_bound.restype = U64
        L.sb_encode_binary_column_device.argtypes = [P, I32, P, U64, P, P, U64, I32, ctypes.POINTER(N.WriteOptionsC), U64,
                                                     P, U64, ctypes.POINTER(U64), ctypes.POINTER(N.PageMetaC), U64,
                                                     ctypes.POINTER(U64)]
        L.sb_encode_binary_column_device.restype = I32
        L._bin_ready = True
    return L


class BinaryOutC(ctypes.Structure):
    _fields_ = [("d_offsets", ctypes.c_void_p), ("d_values", ctypes.c_void_p), ("values_capacity", ctypes.c_uint64),
                ("d_validity", ctypes.c_void_p)]


def encode_binary_column(values: bytes, offsets: np.ndarray, validity=None, nullable: bool = False,
                         options=None, physical_type: int = UTF8, n_threads: int = 0) -> Tuple[bytes, List[PageMeta]]:
    from .write import WriteOptions, _take

    L = _lib()
    options = options or WriteOptions()
    offs = np.ascontiguousarray(offsets, np.int64)
    vals = np.frombuffer(values, np.uint8) if values else np.zeros(1, np.uint8)
    vb = None if validity is None else np.packbits(np.asarray(validity, bool), bitorder="little")
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    metas = ctypes.POINTER(N.PageMetaC)()
    npg = ctypes.c_uint64()
    opts = options.c()
    st = L.sb_encode_binary_column(physical_type, vals.ctypes.data_as(ctypes.c_void_p), len(values),
                                   offs.ctypes.data_as(ctypes.c_void_p),
                                   None if vb is None else vb.ctypes.data_as(ctypes.c_void_p), len(offs) - 1,
                                   int(nullable), ctypes.byref(opts), options.max_page_size or 0, n_threads,
                                   ctypes.byref(out), ctypes.byref(olen), ctypes.byref(metas), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "encode_binary_column")
    pm = [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]
    L.sb_free(metas)
    return _take(out, olen.value), pm


def encode_binary_column_device(values, offsets, validity=None, nullable: bool = False, options=None,
                                physical_type: int = UTF8, ctx: Optional[Context] = None):
    """encode_chunk for one Binary / Utf8 leaf on the GPU
    (sb_encode_binary_column_device): values = the array's whole values buffer
    (device uint8 tensor), offsets = n + 1 absolute positions (device int64
    tensor), validity an optional device bool tensor.  Returns (device uint8
    chunk, page metas), byte-identical to encode_binary_column."""
    import torch

    from .write import WriteOptions

    L = _lib()
    options = options or WriteOptions()
    ctx = resolve_context(ctx, values)
    offsets = offsets.to(dtype=torch.int64).contiguous()
    values = values.contiguous()
    n = offsets.numel() - 1
    vb = None
    if nullable:
        v = (validity.to(device=offsets.device, dtype=torch.bool).reshape(-1) if validity is not None
             else torch.ones(n, dtype=torch.bool, device=offsets.device))
        pad = (-n) % 8
        if pad:
            v = torch.cat([v, torch.zeros(pad, dtype=torch.bool, device=v.device)])
        w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=v.device)
        vb = (v.view(-1, 8).to(torch.uint8) * w).sum(1, dtype=torch.uint8) if n else torch.zeros(
            1, dtype=torch.uint8, device=v.device)
    P = min(options.max_page_size or n, n)
    cap = L.sb_encode_binary_device_bound(physical_type, n, values.numel(), int(nullable), P)
    out = torch.empty(max(cap, 16), dtype=torch.uint8, device=offsets.device)
    npages = (n + P - 1) // P if n else 0
    metas = (N.PageMetaC * max(npages, 1))()
    olen, npg = ctypes.c_uint64(), ctypes.c_uint64()
    opts = options.c()
    st = L.sb_encode_binary_column_device(
        ctx._h, physical_type, ctypes.c_void_p(values.data_ptr()), values.numel(), ctypes.c_void_p(offsets.data_ptr()),
        None if vb is None else ctypes.c_void_p(vb.data_ptr()), n, int(nullable), ctypes.byref(opts), P,
        ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(olen), metas, max(npages, 1), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "encode_binary_column_device: " + ctx.error())
    return out[: olen.value], [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]


class BinaryColumnDecoder:
    """Planned Binary/Utf8 column chunk; values bytes are sized at plan time."""

    def __init__(self, chunk, page_metas: Sequence[PageMeta], physical_type: int = UTF8, nullable: bool = False,
                 ctx: Optional[Context] = None, timing: bool = False):
        import torch

        L = _lib()
        self.ctx = resolve_context(ctx, chunk)
        self.phys = physical_type
        self.nullable = bool(nullable)
        self.chunk = _as_device_bytes(chunk, self.ctx.device)
        self.metas = list(page_metas)
        metas = (N.PageMetaC * max(1, len(self.metas)))(*[N.PageMetaC(m.length, m.num_values) for m in self.metas])
        desc = N.ColumnDescC(physical_type, int(self.nullable))
        h = ctypes.c_void_p()
        st = L.sb_plan_column(self.ctx._h, ctypes.byref(desc), ctypes.c_void_p(self.chunk.data_ptr()),
                              self.chunk.numel(), metas, len(self.metas), ctypes.byref(h))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        self._h = h
        if timing:
            L.sb_plan_enable_timing(h, 1)
        self.num_rows = int(L.sb_plan_num_rows(h))
        self.values_bytes = int(L.sb_plan_values_bytes(h))
        self._torch = torch

    @classmethod
    def for_shard(cls, chunk, page_metas, shard, physical_type: int = UTF8, nullable: bool = False, ctx=None, timing: bool = False):
        """The decoder of one rank's page range (pa_amd.shard_pages): only the
        shard's bytes are planned and decoded; rows start at shard.row_offset
        of the whole column."""
        from .shard import shard_slice

        part, metas = shard_slice(chunk, page_metas, shard)
        dec = cls(part, metas, physical_type, nullable, ctx, timing)
        dec.shard = shard
        return dec

    def alloc_outputs(self):
        torch = self._torch
        dev = f"cuda:{self.ctx.device}"
        odt = torch.int64 if _ow(self.phys) == 8 else torch.int32
        offsets = torch.zeros(self.num_rows + 1, dtype=odt, device=dev)
        values = torch.empty(max(self.values_bytes, 16), dtype=torch.uint8, device=dev)
        validity = None
        if self.nullable:
            validity = torch.zeros(max((self.num_rows + 31) // 32, 1) * 4, dtype=torch.uint8, device=dev)
        return offsets, values, validity

    def decode_async(self, offsets=None, values=None, validity=None):
        if offsets is None:
            offsets, values, validity = self.alloc_outputs()
        out = BinaryOutC(offsets.data_ptr(), values.data_ptr(), values.numel(),
                         validity.data_ptr() if validity is not None else None)
        st = _lib().sb_decode_binary_planned(self.ctx._h, self._h, ctypes.byref(out))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        return offsets, values, validity

    def check(self):
        bad = ctypes.c_int64(-1)
        st = N.lib().sb_plan_status(self.ctx._h, self._h, ctypes.byref(bad))
        if st:
            raise N.StrawboatError(st, self.ctx.error())

    def decode(self, *outs):
        r = self.decode_async(*outs)
        self.check()
        return r

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


def batch_read_binary(chunk, page_metas: Sequence[PageMeta], physical_type: int = UTF8, nullable: bool = False,
                      ctx: Optional[Context] = None):
    """read_binary for one leaf: (offsets, values[:values_bytes], validity|None) device tensors."""
    dec = BinaryColumnDecoder(chunk, page_metas, physical_type, nullable, ctx)
    try:
        o, v, m = dec.decode()
        return o, v[: dec.values_bytes], m
    finally:
        dec.close()
