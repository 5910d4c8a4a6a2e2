"""The file side of the reader (read/reader.rs:148-262): footer and IPC
schema parse, and the file -> HBM staging pipeline in front of the decoders.

`StrawboatFile(path)` is read_meta + infer_schema: its `columns` are the
ColumnMeta of the footer, its `leaves` the schema's leaves in to_leaves
order (one per column).  `upload(col)` stages a column chunk into HBM
through pinned double buffers (sb_file_upload); `decoder(col)` plans the
decoder the leaf's type calls for (the read/deserialize.rs dispatch) on the
uploaded chunk."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _native as N
from .read import _PHYS, ColumnDecoder, ColumnMeta, Context, PageMeta, resolve_context

_DTYPE = {v: k for k, v in _PHYS.items()}

# Schema.fbs Type union tags
ARROW_TYPE = {1: "Null", 2: "Int", 3: "FloatingPoint", 4: "Binary", 5: "Utf8", 6: "Bool", 7: "Decimal", 8: "Date",
              9: "Time", 10: "Timestamp", 11: "Interval", 12: "List", 13: "Struct", 14: "Union",
              15: "FixedSizeBinary", 16: "FixedSizeList", 17: "Map", 18: "Duration", 19: "LargeBinary",
              20: "LargeUtf8", 21: "LargeList"}
LEAF_STRUCT, LEAF_MAP, LEAF_FIXED_SIZE_LIST, LEAF_UNION, LEAF_TOO_DEEP = 1, 2, 4, 8, 16


@dataclass
class Leaf:
    """sb_leaf_info: one leaf column of the schema."""
    name: str
    arrow_type: str
    physical_type: int
    nullable: bool
    depth: int
    list_nullable: List[bool] = field(default_factory=list)
    large_list: List[bool] = field(default_factory=list)
    flags: int = 0
    top_field: int = 0
    struct_mask: int = 0
    map_mask: int = 0
    nest_id: List[int] = field(default_factory=list)

    def nest_kind(self, d: int) -> str:
        if (self.struct_mask >> d) & 1:
            return "struct"
        if (self.map_mask >> d) & 1:
            return "map"
        return "large_list" if self.large_list[d] else "list"


def _leaf(c: N.LeafInfoC) -> Leaf:
    d = min(c.depth, N.MAX_NEST)
    return Leaf(c.name.decode(errors="replace"), ARROW_TYPE.get(c.arrow_type, str(c.arrow_type)), c.physical_type,
                bool(c.nullable), c.depth, [bool(c.list_nullable[i]) for i in range(d)],
                [bool(c.large_list[i]) for i in range(d)], c.flags, c.top_field, c.struct_mask, c.map_mask,
                [int(c.nest_id[i]) for i in range(d)])


def parse_schema(schema_bytes: bytes) -> List[Leaf]:
    """infer_schema's deserialize_schema, flattened to leaves (host only)."""
    L = N.lib()
    buf = bytes(schema_bytes)
    n, nf = ctypes.c_uint64(), ctypes.c_uint64()
    st = L.sb_parse_schema(buf, len(buf), None, 0, ctypes.byref(n), ctypes.byref(nf))
    if st:
        raise N.StrawboatError(st, "schema bytes are not an IPC Schema message")
    arr = (N.LeafInfoC * max(1, n.value))()
    L.sb_parse_schema(buf, len(buf), arr, n.value, ctypes.byref(n), ctypes.byref(nf))
    return [_leaf(arr[i]) for i in range(n.value)]


class StrawboatFile:
    """An open strawboat file: footer metas, schema leaves, staged uploads."""

    def __init__(self, path: str):
        self._h = ctypes.c_void_p()
        st = N.lib().sb_file_open(str(path).encode(), ctypes.byref(self._h))
        if st:
            self._h = None
            raise N.StrawboatError(st, f"cannot read the footer of {path}")
        L = N.lib()
        self.num_columns = int(L.sb_file_num_columns(self._h))
        self._columns: Optional[List[ColumnMeta]] = None
        b, n = ctypes.POINTER(ctypes.c_uint8)(), ctypes.c_uint64()
        self._check(L.sb_file_schema(self._h, ctypes.byref(b), ctypes.byref(n)))
        self.schema_bytes = ctypes.string_at(b, n.value)
        self.leaves: List[Leaf] = parse_schema(self.schema_bytes) if n.value else []

    def _column(self, c: int):
        off, ln, npg = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        pp = ctypes.POINTER(N.PageMetaC)()
        self._check(N.lib().sb_file_column(self._h, c, ctypes.byref(off), ctypes.byref(ln), ctypes.byref(npg),
                                           ctypes.byref(pp)))
        return off.value, ln.value, npg.value, pp

    @property
    def columns(self) -> List[ColumnMeta]:
        """The footer's ColumnMeta list (built on first use)."""
        if self._columns is None:
            cols = []
            for c in range(self.num_columns):
                off, _, npg, pp = self._column(c)
                cols.append(ColumnMeta(off, [PageMeta(pp[i].length, pp[i].num_values) for i in range(npg)]))
            self._columns = cols
        return self._columns

    def _check(self, st):
        if st:
            raise N.StrawboatError(st, N.lib().sb_file_last_error(self._h).decode())

    def upload(self, col: int, ctx: Optional[Context] = None, out=None):
        """Column chunk `col` -> a uint8 device tensor (pinned double-buffered
        H2D; ordered before later work on the context's stream)."""
        import torch

        ctx = resolve_context(ctx, out)
        off, n, _, _ = self._column(col)
        if out is None:
            out = torch.empty(max(1, n), dtype=torch.uint8, device=f"cuda:{ctx.device}")
        elif out.numel() < n or out.dtype != torch.uint8:
            raise N.StrawboatError(N.E_ARG, "upload buffer too small")
        self._check(N.lib().sb_file_upload(ctx._h, self._h, off, n, ctypes.c_void_p(out.data_ptr())))
        return out

    def decoder(self, col: int, ctx: Optional[Context] = None, chunk=None):
        """The decoder of leaf `col` (read/deserialize.rs dispatch: primitive,
        Boolean, Binary / Utf8, List<...>) over its uploaded chunk."""
        from .binary import BINARY, LARGE_BINARY, LARGE_UTF8, UTF8, BinaryColumnDecoder
        from .nested import ListColumnDecoder, NestedColumnDecoder

        if len(self.leaves) != self.num_columns:
            # leaves and column metas pair up one to one (to_leaves order); a
            # mismatch would decode a column with another leaf's type
            raise N.StrawboatError(N.E_OUT_OF_SPEC, f"schema has {len(self.leaves)} leaves but the footer "
                                                    f"{self.num_columns} columns")
        if not 0 <= col < self.num_columns:
            raise N.StrawboatError(N.E_ARG, f"column {col} out of range")
        leaf = self.leaves[col]
        ctx = resolve_context(ctx, chunk)
        if chunk is None:
            chunk = self.upload(col, ctx)
        metas = self.columns[col].pages
        pt = leaf.physical_type
        if leaf.flags & ~(LEAF_STRUCT | LEAF_MAP) or not pt:
            raise N.StrawboatError(N.E_NYI, f"leaf {leaf.name}: {leaf.arrow_type} (flags {leaf.flags}) has no page path here")
        binary = pt in (BINARY, LARGE_BINARY, UTF8, LARGE_UTF8)
        dtype = _DTYPE.get(pt, np.uint8)
        if leaf.depth == 0:
            if binary:
                return BinaryColumnDecoder(chunk, metas, pt, leaf.nullable, ctx=ctx)
            return ColumnDecoder(chunk, metas, dtype, leaf.nullable, ctx=ctx)
        lists = [leaf.large_list[d] for d in range(leaf.depth) if not (leaf.struct_mask >> d) & 1]
        large = bool(lists and lists[0])
        if any(x != large for x in lists):
            raise N.StrawboatError(N.E_NYI, f"leaf {leaf.name}: mixed List / LargeList levels")
        if leaf.depth == 1 and not leaf.struct_mask and not binary and pt != N.BOOLEAN:
            return ListColumnDecoder(chunk, metas, dtype, leaf.list_nullable[0], leaf.nullable, ctx=ctx, large=large)
        return NestedColumnDecoder(chunk, metas, dtype, leaf.list_nullable, leaf.nullable, ctx=ctx, large=large,
                                   physical_type=pt, struct_mask=leaf.struct_mask)

    def field(self, top: int):
        """The pa_amd.Field tree of top-level field `top`, rebuilt from its
        leaves' nest chains (the nest ids group the leaves of one struct or
        map) -> (Field, [leaf column indices])."""
        from .nested import Field

        cols = [c for c, l in enumerate(self.leaves) if l.top_field == top]
        if not cols:
            raise N.StrawboatError(N.E_ARG, f"no leaf columns for field {top}")

        def build(cs, d):
            first = self.leaves[cs[0]]
            if d == first.depth:
                assert len(cs) == 1
                return Field.leaf(first.physical_type, first.nullable, first.name) if first.physical_type not in _DTYPE \
                    else Field.leaf(_DTYPE[first.physical_type], first.nullable, first.name)
            kind = first.nest_kind(d)
            groups = []  # children: consecutive leaves sharing the nest id at d + 1 (or a leaf at d + 1)
            for c in cs:
                lf = self.leaves[c]
                key = lf.nest_id[d + 1] if lf.depth > d + 1 else ("leaf", c)
                if not groups or groups[-1][0] != key:
                    groups.append((key, []))
                groups[-1][1].append(c)
            kids = [build(g, d + 1) for _, g in groups]
            if kind != "struct" and len(kids) != 1:
                raise N.StrawboatError(N.E_OUT_OF_SPEC, "a list nest with several children")
            return Field(kind, bool(first.list_nullable[d]), kids)

        if any(self.leaves[c].depth > N.MAX_NEST or self.leaves[c].flags & ~(LEAF_STRUCT | LEAF_MAP) for c in cols):
            raise N.StrawboatError(N.E_NYI, f"field {top} has no page path here")
        return build(cols, 0), cols

    def read_field(self, top: int, ctx: Optional[Context] = None):
        """batch_read_array for top-level field `top` (read/batch_read.rs:
        190-209): a primitive field -> its column decoder's outputs, a nested
        one -> a pa_amd.DeviceArray tree (FieldDecoder over its leaves)."""
        from .nested import FieldDecoder

        fld, cols = self.field(top)
        ctx = resolve_context(ctx, None)
        if fld.kind == "leaf":
            dec = self.decoder(cols[0], ctx)
            try:
                return dec.decode()
            finally:
                dec.close()
        dec = FieldDecoder(fld, [(self.upload(c, ctx), self.columns[c].pages) for c in cols], ctx)
        try:
            return dec.decode()
        finally:
            dec.close()

    def close(self):
        if getattr(self, "_h", None):
            N.lib().sb_file_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
