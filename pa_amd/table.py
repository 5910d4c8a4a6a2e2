"""Several leaves of a chunk decoded as one plan (sb_plan_column_at).

The reference decodes a chunk's leaves one by one (column_iter_to_arrays /
batch_read_array per leaf, read/deserialize.rs:237-253,
read/batch_read.rs:190-209).  They are independent, and on the GPU a
column of ~1000 pages is too small a launch to fill 256 CUs: the fixed-width
(and Boolean) leaves of one type and nullability whose chunks lie back to
back -- as a file's column chunks do -- decode here as ONE plan, each leaf at
its own row base (a multiple of 32, so its validity stays word-aligned), and
one launch sequence replaces one per leaf.  Each leaf's arrays are views of
the group's outputs, byte-identical to a per-leaf ColumnDecoder.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .read import Context, PageMeta, _as_device_bytes, physical_type, resolve_context


class ColumnGroupDecoder:
    """columns: [(chunk, page metas)] of leaves with one dtype and
    nullability; their chunks are concatenated on the device (the bytes a
    file holds back to back) and planned once."""

    def __init__(self, columns: Sequence[Tuple[object, Sequence[PageMeta]]], dtype, nullable: bool,
                 ctx: Optional[Context] = None):
        import torch

        cols = list(columns)
        if not cols:
            raise N.StrawboatError(N.E_ARG, "no columns")
        self.ctx = resolve_context(ctx, cols[0][0])
        self.dtype = np.dtype(dtype)
        self.nullable = bool(nullable)
        parts = [_as_device_bytes(c, self.ctx.device) for c, _ in cols]
        self.chunk = torch.cat(parts) if len(parts) > 1 else parts[0]
        metas, rows_at, self.bases, self.rows = [], [], [], []
        base = 0
        for _, ms in cols:
            self.bases.append(base)
            r = base
            for m in ms:
                metas.append(m)
                rows_at.append(r)
                r += m.num_values
            self.rows.append(r - base)
            base = (r + 31) // 32 * 32
        self.num_rows = base
        cm = (N.PageMetaC * max(1, len(metas)))(*[N.PageMetaC(m.length, m.num_values) for m in metas])
        ro = (ctypes.c_uint64 * max(1, len(rows_at)))(*rows_at)
        desc = N.ColumnDescC(physical_type(self.dtype), int(self.nullable))
        h = ctypes.c_void_p()
        st = N.lib().sb_plan_column_at(self.ctx._h, ctypes.byref(desc), ctypes.c_void_p(self.chunk.data_ptr()),
                                       self.chunk.numel(), cm, len(metas), ro, ctypes.byref(h))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        self._h = h
        self._torch = torch

    def alloc_outputs(self):
        torch = self._torch
        dev = f"cuda:{self.ctx.device}"
        nwords = max((self.num_rows + 31) // 32, 1)
        if self.dtype == np.bool_:
            values = torch.zeros(nwords * 4, dtype=torch.uint8, device=dev)
        else:
            tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[self.dtype.itemsize]
            values = torch.empty(max(self.num_rows, 1), dtype=tdt, device=dev)
        validity = torch.zeros(nwords * 4, dtype=torch.uint8, device=dev) if self.nullable else None
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

    def column(self, i: int, values, validity=None):
        """Leaf i's (values, validity|None) views of the group's outputs
        (Boolean values: its bitmap words, like the validity)."""
        b, n = self.bases[i], self.rows[i]
        if self.dtype == np.bool_:
            v = values[b // 8:(b + n + 31) // 32 * 4]
        else:
            v = values[b:b + n]
        m = validity[b // 8:(b + n + 31) // 32 * 4] if validity is not None else None
        return v, m

    def decode(self, values=None, validity=None) -> List[Tuple[object, object]]:
        v, m = self.decode_async(values, validity)
        self.check()
        return [self.column(i, v, m) for i in range(len(self.bases))]

    def close(self):
        if getattr(self, "_h", None):
            N.lib().sb_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
