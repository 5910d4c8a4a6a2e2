"""Page-at-a-time reading (column_iter_to_arrays, read/deserialize.rs:237-253)
decoded in page ranges, and host materialisation of decoded arrays
(batch_read_array returns host arrays, read/batch_read.rs:190-209).

The reference's iterator decodes one page per next() and returns the arrays
of pages 0..k-1 before the error of a bad page k.  Here a next() that finds
no decoded page left reads the next `range_pages` pages of every leaf reader,
stages them into HBM (one copy per leaf) and decodes them in one launch --
any page range of a chunk is itself a valid chunk -- so memory is bounded by
the range.  If the range fails, its pages are decoded one by one so the
arrays before the bad page come back first, then its error.  The Rust shim's
compat::column_iter_to_arrays follows the same protocol.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Iterator, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .binary import BINARY, LARGE_BINARY, LARGE_UTF8, UTF8, BinaryColumnDecoder
from .nested import DeviceArray, Field, FieldDecoder, HostArray
from .read import ColumnDecoder, Context, PageMeta, resolve_context

_BINARY = (BINARY, UTF8, LARGE_BINARY, LARGE_UTF8)


def decode_columns(fld: Field, columns, ctx: Optional[Context] = None) -> DeviceArray:
    """batch_read_array for any field: a flat leaf (one column) or a nested
    field (one column per leaf, to_leaves order) -> DeviceArray."""
    if fld.kind != "leaf":
        dec = FieldDecoder(fld, columns, ctx)
        try:
            return dec.decode()
        finally:
            dec.close()
    (chunk, metas), = columns
    if fld.physical_type in _BINARY:
        dec = BinaryColumnDecoder(chunk, metas, fld.physical_type, fld.nullable, ctx)
        try:
            o, v, m = dec.decode()
            return DeviceArray("leaf", dec.num_rows, m, values=(o, v))
        finally:
            dec.close()
    dtype = np.bool_ if fld.physical_type == N.BOOLEAN else fld.dtype
    dec = ColumnDecoder(chunk, metas, dtype, fld.nullable, ctx)
    try:
        v, m = dec.decode()
        return DeviceArray("leaf", dec.num_rows, m, values=v)
    finally:
        dec.close()


def _bits(t, b: int, n: int) -> np.ndarray:
    """Bits [b, b + n) of a device bitmap as bools (one D2H copy of their bytes)."""
    raw = t[b // 8:(b + n + 7) // 8 + 1].cpu().numpy().view(np.uint8)
    return np.unpackbits(raw, bitorder="little")[b % 8:b % 8 + n].astype(bool)


def _offsets(t, b: int, e: int) -> np.ndarray:
    return t[b:e + 1].cpu().numpy().astype(np.int64)


def to_host(fld: Field, arr: DeviceArray, b: int = 0, e: Optional[int] = None) -> HostArray:
    """Rows [b, e) of a decoded array as a host array of the reference's shape
    (a HostArray tree): values, offsets rebased to 0, validity per slot; a
    list / map carries the child slots its rows reach."""
    e = arr.length if e is None else e
    n = e - b
    valid = None if arr.validity is None else _bits(arr.validity, b, n)
    if fld.kind == "leaf":
        if fld.physical_type in _BINARY:
            o = _offsets(arr.values[0], b, e)
            data = arr.values[1][int(o[0]):int(o[-1])].cpu().numpy().tobytes()
            return HostArray("leaf", n, valid, values=(o - o[0], data))
        if fld.physical_type == N.BOOLEAN:
            return HostArray("leaf", n, valid, values=_bits(arr.values, b, n))
        w = fld.dtype.itemsize
        raw = arr.values.view(-1).view(__import__("torch").uint8)[b * w:e * w].cpu().numpy()
        return HostArray("leaf", n, valid, values=raw.view(fld.dtype).copy())
    if fld.kind == "struct":
        kids = [to_host(c, x, b, e) for c, x in zip(fld.children, arr.children)]
        return HostArray("struct", n, valid, children=kids)
    o = _offsets(arr.offsets, b, e)
    child = to_host(fld.children[0], arr.children[0], int(o[0]), int(o[-1]))
    return HostArray(fld.kind, n, valid, offsets=o - o[0], children=[child])


@dataclass
class PageArray:
    """One page's array: rows [offset, offset + length) of a decoded page
    range (arrow2's sliced arrays share their buffers the same way)."""
    field: Field
    data: DeviceArray
    offset: int
    length: int

    def to_host(self) -> HostArray:
        return to_host(self.field, self.data, self.offset, self.offset + self.length)


def _page_rows(fld: Field, num_values: int, page: bytes) -> int:
    if fld.kind == "leaf":
        return num_values
    if len(page) < 4:
        raise N.StrawboatError(N.E_OUT_OF_SPEC, "nested page shorter than its header")
    return int.from_bytes(page[:4], "little")  # write_nested_validity's u32 rows


def iter_page_arrays(readers: Sequence[Iterable[Tuple[int, bytes]]], fld: Field, ctx: Optional[Context] = None,
                     range_pages: int = 64) -> Iterator[PageArray]:
    """column_iter_to_arrays over one reader per leaf column (each yields
    (num_values, page bytes), e.g. pa_amd.NativeReader): one PageArray per
    page, in page order, decoded `range_pages` pages per launch; a bad page
    raises after the arrays of the pages before it."""
    ctx = resolve_context(ctx)
    its = [iter(r) for r in readers]
    while True:
        chunks, metas, rows, err = [], [], None, None
        want = range_pages
        for k, it in enumerate(its):
            buf, ms, rs = bytearray(), [], []
            while len(ms) < want:
                try:
                    nv, page = next(it)
                except StopIteration:
                    break
                except N.StrawboatError as ex:
                    err = ex
                    break
                try:
                    rs.append(_page_rows(fld, nv, page))
                except N.StrawboatError as ex:
                    err = ex
                    break
                ms.append(PageMeta(len(page), nv))
                buf += page
            if k == 0:
                want, rows = len(ms), rs
            elif rs != rows[:len(rs)]:  # StructIterator zips page k of every child (struct_.rs:63-85)
                err = err or N.StrawboatError(N.E_OUT_OF_SPEC, "leaf columns page different rows")
            elif len(ms) < want and err is None:
                err = N.StrawboatError(N.E_OUT_OF_SPEC, "leaf columns hold different pages")
            if err is not None:
                want = min(want, len(ms))
            chunks.append(bytes(buf))
            metas.append(ms)
        n = want
        for k in range(len(chunks)):  # every leaf keeps the pages all leaves could read
            metas[k] = metas[k][:n]
            chunks[k] = chunks[k][:sum(m.length for m in metas[k])]
        rows = rows[:n]
        if n:
            yield from _decode_range(fld, chunks, metas, rows, ctx)
        if err is not None:
            raise err
        if n < range_pages:
            return


def _decode_range(fld, chunks, metas, rows, ctx) -> Iterator[PageArray]:
    try:
        data = decode_columns(fld, list(zip(chunks, metas)), ctx)
        if data.length != sum(rows):
            raise N.StrawboatError(N.E_OUT_OF_SPEC, f"pages hold {sum(rows)} rows, the decode {data.length}")
    except N.StrawboatError:
        out = []
        for p in range(len(rows)):  # find the bad page: the pages before it come back first
            one = []
            for c, m in zip(chunks, metas):
                s = sum(x.length for x in m[:p])
                one.append((c[s:s + m[p].length], [m[p]]))
            try:
                d = decode_columns(fld, one, ctx)
            except N.StrawboatError:
                yield from out
                raise
            out.append(PageArray(fld, d, 0, rows[p]))
        yield from out
        return
    first = 0
    for r in rows:
        yield PageArray(fld, data, first, r)
        first += r
