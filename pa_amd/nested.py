"""Nested columns: List<primitive> (one list level over a primitive leaf),
any List / Map / Struct chain over a leaf, and whole Struct / Map fields.

Reference (b41sh/pa @ 2025-01-17):
  write_nested / write_nested_validity   src/write/serialize.rs:133-146, 217-232
  read_validity_nested                   src/read/read_basic.rs:65-173
  read_nested_integer / _double          src/read/array/integer.rs:240-261, double.rs
  create_list                            src/read/array/list.rs:48
  deserialize_nested (InitNested chain)  src/read/deserialize.rs:140-233
  create_struct / MapIterator            src/read/array/struct_.rs:101-114, map.rs
  read_nested (batch)                    src/read/batch_read.rs:67-180
  encode_chunk (paging by top-level rows) src/write/common.rs:49-119

encode_list_column -> sb_encode_list_column (host encoder)
ListColumnDecoder  -> sb_plan_list_column (device sizing) + sb_decode_list_planned
batch_read_list    -> one ListArray per column: (offsets, list validity, values, leaf validity)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N
from .binary import BINARY, LARGE_BINARY, LARGE_UTF8, UTF8
from .read import Context, PageMeta, resolve_context, physical_type, _as_device_bytes


class ListDescC(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("list_nullable", ctypes.c_int32),
                ("item_nullable", ctypes.c_int32), ("offset_width", ctypes.c_int32)]


class ListOutC(ctypes.Structure):
    _fields_ = [("d_offsets", ctypes.c_void_p), ("d_list_validity", ctypes.c_void_p), ("d_values", ctypes.c_void_p),
                ("d_leaf_validity", ctypes.c_void_p)]


def _lib():
    L = N.lib()
    if not getattr(L, "_list_ready", False):
        P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
        PU8 = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8))
        L.sb_encode_list_column.argtypes = [I32, P, P, I32, P, P, I32, U64, ctypes.POINTER(N.WriteOptionsC), U64, I32,
                                            PU8, ctypes.POINTER(U64), ctypes.POINTER(ctypes.POINTER(N.PageMetaC)),
                                            ctypes.POINTER(U64)]
        L.sb_encode_list_column.restype = I32
        L.sb_plan_list_column.argtypes = [P, ctypes.POINTER(ListDescC), P, U64, ctypes.POINTER(N.PageMetaC), U64,
                                          ctypes.POINTER(ctypes.c_void_p)]
        L.sb_plan_list_column.restype = I32
        L.sb_plan_num_leaves.argtypes = [P]
        L.sb_plan_num_leaves.restype = U64
        L.sb_decode_list_planned.argtypes = [P, P, ctypes.POINTER(ListOutC)]
        L.sb_decode_list_planned.restype = I32
        L._list_ready = True
    return L


def encode_list_column(offsets: np.ndarray, child: np.ndarray, list_validity=None, child_validity=None,
                       list_nullable: bool = False, item_nullable: bool = False, options=None,
                       n_threads: int = 0) -> Tuple[bytes, List[PageMeta]]:
    """encode_chunk for one List<T> leaf: pages of options.max_page_size
    top-level rows; PageMeta.num_values = the page's level count."""
    from .write import WriteOptions, _take

    L = _lib()
    options = options or WriteOptions()
    offs = np.ascontiguousarray(offsets, np.int64)
    child = np.ascontiguousarray(child)
    if len(child) == 0:
        child = np.zeros(1, child.dtype)
    lvb = None if list_validity is None else np.packbits(np.asarray(list_validity, bool), bitorder="little")
    cvb = None if child_validity is None else np.packbits(np.asarray(child_validity, bool), bitorder="little")
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_uint64()
    metas = ctypes.POINTER(N.PageMetaC)()
    npg = ctypes.c_uint64()
    opts = options.c()
    vp = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    st = L.sb_encode_list_column(physical_type(child.dtype), vp(offs), vp(lvb), int(list_nullable), vp(child), vp(cvb),
                                 int(item_nullable), len(offs) - 1, ctypes.byref(opts), options.max_page_size or 0,
                                 n_threads, ctypes.byref(out), ctypes.byref(olen), ctypes.byref(metas),
                                 ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "encode_list_column")
    pm = [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]
    L.sb_free(metas)
    return _take(out, olen.value), pm


def encode_list_column_device(offsets, child, list_validity=None, child_validity=None, list_nullable: bool = False,
                              item_nullable: bool = False, options=None, ctx=None):
    """encode_chunk for one List<T> leaf on the GPU
    (sb_encode_list_column_device): offsets (n + 1 absolute int64
    positions), child, list_validity (over the rows) and child_validity (over
    the child values) are device tensors; returns (device uint8 tensor of the
    column chunk, page metas), byte-identical to encode_list_column with the
    same options."""
    import torch

    from .read import resolve_context
    from .write import WriteOptions

    L = _lib()
    options = options or WriteOptions()
    ctx = resolve_context(ctx, child)
    offs = offsets.to(torch.int64).contiguous()
    child = child.contiguous()
    n = offs.numel() - 1
    tdt = {torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32, torch.int64: np.int64,
           torch.uint8: np.uint8, torch.uint16: np.uint16, torch.uint32: np.uint32, torch.uint64: np.uint64,
           torch.float32: np.float32, torch.float64: np.float64}[child.dtype]
    phys = physical_type(np.dtype(tdt))

    def pack(bits, m):  # bool device tensor -> LSB-first bitmap bytes (at least one byte)
        bits = bits.to(device=child.device, dtype=torch.bool).reshape(-1)
        pad = (-m) % 8
        if pad:
            bits = torch.cat([bits, torch.zeros(pad, dtype=torch.bool, device=bits.device)])
        if not m:
            return torch.zeros(1, dtype=torch.uint8, device=child.device)
        w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=child.device)
        return (bits.view(-1, 8).to(torch.uint8) * w).sum(1, dtype=torch.uint8)

    nc = child.numel()
    lvb = pack(list_validity if list_validity is not None else torch.ones(n, dtype=torch.bool), n) \
        if list_nullable else None
    cvb = pack(child_validity if child_validity is not None else torch.ones(nc, dtype=torch.bool), nc) \
        if item_nullable else None
    if nc == 0:
        child = torch.zeros(1, dtype=child.dtype, device=child.device)
    P = min(options.max_page_size or n, n)
    n_child = int(offs[-1].item() - offs[0].item()) if n else 0
    cap = L.sb_encode_list_device_bound(phys, n, n_child, int(item_nullable), P)
    out = torch.empty(max(cap, 16), dtype=torch.uint8, device=child.device)
    npages = (n + P - 1) // P if n else 0
    metas = (N.PageMetaC * max(npages, 1))()
    olen, npg = ctypes.c_uint64(), ctypes.c_uint64()
    opts = options.c()
    vp = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = L.sb_encode_list_column_device(ctx._h, phys, vp(offs), vp(lvb), int(list_nullable), vp(child), vp(cvb),
                                        int(item_nullable), n, ctypes.byref(opts), P, vp(out), out.numel(),
                                        ctypes.byref(olen), metas, max(npages, 1), ctypes.byref(npg))
    if st:
        raise N.StrawboatError(st, "encode_list_column_device: " + ctx.error())
    return out[: olen.value], [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]


class ListColumnDecoder:
    """A planned List<T> column chunk: rows and leaves are sized on the device
    at plan time; decode() re-runs the sizing pass, the levels pass and the
    values decode into caller- or self-allocated device buffers."""

    def __init__(self, chunk, page_metas: Sequence[PageMeta], dtype, list_nullable: bool, item_nullable: bool,
                 ctx: Optional[Context] = None, large: bool = False, timing: bool = False):
        import torch

        self._torch = torch
        self.ctx = resolve_context(ctx, chunk)
        self.dtype = np.dtype(dtype)
        self.list_nullable, self.item_nullable = bool(list_nullable), bool(item_nullable)
        self.offset_width = 8 if large else 4
        self.chunk = _as_device_bytes(chunk, self.ctx.device)
        self.metas = list(page_metas)
        L = _lib()
        metas = (N.PageMetaC * max(1, len(self.metas)))(*[N.PageMetaC(m.length, m.num_values) for m in self.metas])
        desc = ListDescC(physical_type(self.dtype), int(self.list_nullable), int(self.item_nullable), self.offset_width)
        h = ctypes.c_void_p()
        st = L.sb_plan_list_column(self.ctx._h, ctypes.byref(desc), ctypes.c_void_p(self.chunk.data_ptr()),
                                   self.chunk.numel(), metas, len(self.metas), ctypes.byref(h))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        self._h = h
        if timing:
            L.sb_plan_enable_timing(h, 1)
        self.num_rows = int(L.sb_plan_num_rows(h))
        self.num_leaves = int(L.sb_plan_num_leaves(h))

    @classmethod
    def for_shard(cls, chunk, page_metas, shard, dtype, list_nullable: bool, item_nullable: bool, ctx=None, large: bool = False, timing: bool = False):
        """The decoder of one rank's page range (pa_amd.shard_pages): only the
        shard's bytes are planned and decoded; rows start at shard.row_offset
        of the whole column."""
        from .shard import shard_slice

        part, metas = shard_slice(chunk, page_metas, shard)
        dec = cls(part, metas, dtype, list_nullable, item_nullable, ctx, large, timing)
        dec.shard = shard
        return dec

    def alloc_outputs(self):
        torch = self._torch
        dev = f"cuda:{self.ctx.device}"
        odt = torch.int64 if self.offset_width == 8 else torch.int32
        offsets = torch.empty(self.num_rows + 1, dtype=odt, device=dev)
        tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[self.dtype.itemsize]
        values = torch.empty(max(self.num_leaves, 1), dtype=tdt, device=dev)
        bm = lambda n: torch.empty(max((n + 31) // 32, 1) * 4, dtype=torch.uint8, device=dev)  # noqa: E731
        lv = bm(self.num_rows) if self.list_nullable else None
        fv = bm(self.num_leaves) if self.item_nullable else None
        return offsets, lv, values, fv

    def decode_async(self, offsets=None, list_validity=None, values=None, leaf_validity=None):
        if offsets is None:
            offsets, list_validity, values, leaf_validity = self.alloc_outputs()
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        out = ListOutC(p(offsets), p(list_validity), p(values), p(leaf_validity))
        st = _lib().sb_decode_list_planned(self.ctx._h, self._h, ctypes.byref(out))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        return offsets, list_validity, values, leaf_validity

    def check(self):
        bad = ctypes.c_int64(-1)
        st = N.lib().sb_plan_status(self.ctx._h, self._h, ctypes.byref(bad))
        if st:
            raise N.StrawboatError(st, self.ctx.error())

    def decode(self, *bufs):
        r = self.decode_async(*bufs)
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


def batch_read_list(chunk, page_metas: Sequence[PageMeta], dtype, list_nullable: bool, item_nullable: bool,
                    ctx: Optional[Context] = None, large: bool = False):
    """batch_read_array for a List<T> leaf -> device tensors
    (offsets, list validity bitmap|None, values, leaf validity bitmap|None)."""
    dec = ListColumnDecoder(chunk, page_metas, dtype, list_nullable, item_nullable, ctx, large)
    try:
        return dec.decode()
    finally:
        dec.close()


MAX_NEST = 4


class NestedDescC(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("depth", ctypes.c_int32),
                ("list_nullable", ctypes.c_int32 * MAX_NEST), ("item_nullable", ctypes.c_int32),
                ("offset_width", ctypes.c_int32), ("struct_mask", ctypes.c_int32)]


class NestedOutC(ctypes.Structure):
    _fields_ = [("d_offsets", ctypes.c_void_p * MAX_NEST), ("d_validity", ctypes.c_void_p * MAX_NEST),
                ("d_values", ctypes.c_void_p), ("d_leaf_validity", ctypes.c_void_p), ("d_leaf_offsets", ctypes.c_void_p),
                ("values_capacity", ctypes.c_uint64)]


def _nested_lib():
    L = N.lib()
    if not getattr(L, "_nested_ready", False):
        P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
        L.sb_plan_nested_column.argtypes = [P, ctypes.POINTER(NestedDescC), P, U64, ctypes.POINTER(N.PageMetaC), U64,
                                            ctypes.POINTER(ctypes.c_void_p)]
        L.sb_plan_nested_column.restype = I32
        L.sb_plan_nested_count.argtypes = [P, I32]
        L.sb_plan_nested_count.restype = U64
        L.sb_decode_nested_planned.argtypes = [P, P, ctypes.POINTER(NestedOutC)]
        L.sb_decode_nested_planned.restype = I32
        L.sb_plan_values_bytes.argtypes = [P]
        L.sb_plan_values_bytes.restype = U64
        L._nested_ready = True
    return L


class NestedColumnDecoder:
    """A leaf under len(list_nullable) nests (List<List<T>>, List<Struct<..>>,
    Map<K, V> ..., nest 0 outermost; bit d of struct_mask marks a Struct
    nest): read_validity_nested in its general form (read_basic.rs:95-164)
    + create_list per list nest.  decode() -> (offsets per nest | None for
    struct nests, validity per nest | None, values, leaf validity | None)
    device tensors; values is a bitmap for a Boolean leaf (dtype bool) and
    (leaf offsets, value bytes) for a Binary / Utf8 leaf
    (physical_type=pa_amd.UTF8 ...)."""

    def __init__(self, chunk, page_metas: Sequence[PageMeta], dtype, list_nullable, item_nullable: bool,
                 ctx: Optional[Context] = None, large: bool = False, physical_type: Optional[int] = None,
                 struct_mask: int = 0):
        import torch

        self._torch = torch
        self.ctx = resolve_context(ctx, chunk)
        self.dtype = np.dtype(dtype)
        self.list_nullable = tuple(bool(x) for x in list_nullable)
        self.depth = len(self.list_nullable)
        if not 1 <= self.depth <= MAX_NEST:
            raise N.StrawboatError(N.E_NYI, f"nesting depth {self.depth} not supported")
        self.item_nullable = bool(item_nullable)
        self.struct_mask = int(struct_mask)
        self.offset_width = 8 if large else 4
        self.chunk = _as_device_bytes(chunk, self.ctx.device)
        self.metas = list(page_metas)
        L = _nested_lib()
        metas = (N.PageMetaC * max(1, len(self.metas)))(*[N.PageMetaC(m.length, m.num_values) for m in self.metas])
        ln = (ctypes.c_int32 * MAX_NEST)(*([int(x) for x in self.list_nullable] + [0] * (MAX_NEST - self.depth)))
        self.phys = physical_type if physical_type is not None else globals()["physical_type"](self.dtype)
        self.binary = self.phys in (BINARY, UTF8, LARGE_BINARY, LARGE_UTF8)
        desc = NestedDescC(self.phys, self.depth, ln, int(self.item_nullable), self.offset_width, self.struct_mask)
        h = ctypes.c_void_p()
        st = L.sb_plan_nested_column(self.ctx._h, ctypes.byref(desc), ctypes.c_void_p(self.chunk.data_ptr()),
                                     self.chunk.numel(), metas, len(self.metas), ctypes.byref(h))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        self._h = h
        self.counts = [int(L.sb_plan_nested_count(h, d)) for d in range(self.depth + 1)]
        self.values_bytes = int(L.sb_plan_values_bytes(h))

    def alloc_outputs(self):
        torch = self._torch
        dev = f"cuda:{self.ctx.device}"
        odt = torch.int64 if self.offset_width == 8 else torch.int32
        bm = lambda n: torch.empty(max((n + 31) // 32, 1) * 4, dtype=torch.uint8, device=dev)  # noqa: E731
        offs = [None if self.is_struct(d) else torch.empty(self.counts[d] + 1, dtype=odt, device=dev)
                for d in range(self.depth)]
        valid = [bm(self.counts[d]) if self.list_nullable[d] else None for d in range(self.depth)]
        nleaf = self.counts[self.depth]
        if self.binary:
            lo = torch.zeros(nleaf + 1, dtype=torch.int64 if self.phys in (LARGE_BINARY, LARGE_UTF8) else torch.int32,
                             device=dev)
            values = (lo, torch.empty(max(self.values_bytes, 16), dtype=torch.uint8, device=dev))
        elif self.phys == N.BOOLEAN:
            values = torch.zeros(max((nleaf + 31) // 32, 1) * 4, dtype=torch.uint8, device=dev)
        else:
            tdt = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[self.dtype.itemsize]
            values = torch.empty(max(nleaf, 1), dtype=tdt, device=dev)
        leaf = bm(nleaf) if self.item_nullable else None
        return offs, valid, values, leaf

    def is_struct(self, d: int) -> bool:
        return bool((self.struct_mask >> d) & 1)

    def decode(self, outs=None):
        offs, valid, values, leaf = outs or self.alloc_outputs()
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        o = NestedOutC()
        for d in range(self.depth):
            o.d_offsets[d] = p(offs[d])
            o.d_validity[d] = p(valid[d])
        if self.binary:
            o.d_leaf_offsets = p(values[0])
            o.d_values = p(values[1])
            o.values_capacity = values[1].numel()
        else:
            o.d_values = p(values)
        o.d_leaf_validity = p(leaf)
        L = _nested_lib()
        st = L.sb_decode_nested_planned(self.ctx._h, self._h, ctypes.byref(o))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        bad = ctypes.c_int64(-1)
        st = N.lib().sb_plan_status(self.ctx._h, self._h, ctypes.byref(bad))
        if st:
            raise N.StrawboatError(st, self.ctx.error())
        return offs, valid, values, leaf

    def close(self):
        if getattr(self, "_h", None):
            N.lib().sb_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass



# ---- whole nested fields: Struct / Map / List trees over several leaves -------
@dataclass
class Field:
    """An arrow2 Field restricted to the codec path (the read/deserialize.rs
    dispatch).  kind: "list", "large_list", "map", "struct" or "leaf"; a map's
    one child is its entries struct (key, value); a leaf carries its
    physical type (pa_amd.read.physical_type(dtype), BOOLEAN, BINARY / UTF8 /
    LARGE_*) and, for fixed-width leaves, the numpy dtype."""
    kind: str
    nullable: bool
    children: List["Field"] = field(default_factory=list)
    physical_type: int = 0
    dtype: object = None
    name: str = ""

    @staticmethod
    def leaf(dtype_or_type, nullable: bool, name: str = "") -> "Field":
        if isinstance(dtype_or_type, (int, np.integer)):
            return Field("leaf", nullable, physical_type=int(dtype_or_type), name=name)
        dt = np.dtype(dtype_or_type)
        return Field("leaf", nullable, physical_type=physical_type(dt), dtype=dt, name=name)

    @staticmethod
    def list(child: "Field", nullable: bool, large: bool = False, name: str = "") -> "Field":
        return Field("large_list" if large else "list", nullable, [child], name=name)

    @staticmethod
    def struct(children, nullable: bool, name: str = "") -> "Field":
        return Field("struct", nullable, list(children), name=name)

    @staticmethod
    def map(key: "Field", value: "Field", nullable: bool, name: str = "") -> "Field":
        return Field("map", nullable, [Field("struct", False, [key, value], name="entries")], name=name)

    def n_columns(self) -> int:
        """arrow2 n_columns: the leaf columns under this field."""
        return 1 if self.kind == "leaf" else sum(c.n_columns() for c in self.children)

    def leaf_paths(self, prefix=()):
        """to_leaves order (write/common.rs:66-71): depth first."""
        path = prefix + (self,)
        if self.kind == "leaf":
            return [path]
        return [p for c in self.children for p in c.leaf_paths(path)]


@dataclass
class DeviceArray:
    """A decoded nested array in HBM.  validity: a 32-bit-word Arrow bitmap
    (uint8 tensor) or None; list / map: offsets and children[0]; struct:
    children; leaf: values (fixed width: a typed tensor; Boolean: a bitmap;
    Binary / Utf8: (offsets, bytes))."""
    kind: str
    length: int
    validity: object = None
    offsets: object = None
    children: List["DeviceArray"] = field(default_factory=list)
    values: object = None


def init_chain(path):
    """deserialize_nested's InitNested chain for one leaf path
    (read/deserialize.rs:140-233) -> (nest nullable, struct_mask, leaf
    nullable, large list offsets)."""
    nulls, mask, large = [], 0, set()
    for d, f in enumerate(path[:-1]):
        nulls.append(bool(f.nullable))
        if f.kind == "struct":
            mask |= 1 << d
        else:
            large.add(f.kind == "large_list")
    if len(large) > 1:
        raise N.StrawboatError(N.E_NYI, "List and LargeList nests in one chain")
    return tuple(nulls), mask, bool(path[-1].nullable), large == {True}


class FieldDecoder:
    """batch_read_array / column_iter_to_arrays for a nested field
    (read/batch_read.rs:67-180, read/deserialize.rs:140-233): one
    NestedColumnDecoder per leaf column (to_leaves order), each with the
    leaf's InitNested chain; decode() assembles the array tree, a nest's
    offsets and validity taken from the LAST leaf under it (create_list /
    create_map / create_struct pop the last child's NestedState,
    read/array/struct_.rs:101-114).  Every leaf column of a struct must hold
    the same rows per page (the writer pages all leaves of a field alike,
    write/common.rs:73-100); a leaf whose nest counts disagree is OutOfSpec."""

    def __init__(self, fld: Field, columns, ctx: Optional[Context] = None):
        if fld.kind == "leaf":
            raise N.StrawboatError(N.E_ARG, "a primitive field is not nested: use ColumnDecoder")
        self.field = fld
        self.paths = fld.leaf_paths()
        if len(columns) != len(self.paths):
            raise N.StrawboatError(N.E_ARG, f"{len(self.paths)} leaves but {len(columns)} columns")
        self.ctx = resolve_context(ctx, columns[0][0] if columns else None)
        self.decoders = []
        try:
            for path, (chunk, metas) in zip(self.paths, columns):
                nulls, mask, leaf_null, large = init_chain(path)
                lf = path[-1]
                dtype = lf.dtype if lf.dtype is not None else np.uint8
                self.decoders.append(NestedColumnDecoder(chunk, metas, dtype, nulls, leaf_null, self.ctx, large=large,
                                                         physical_type=lf.physical_type, struct_mask=mask))
        except Exception:
            self.close()
            raise
        self._check_counts(self.field, self.decoders, 0)
        self.num_rows = self.decoders[0].counts[0]

    def _check_counts(self, f: Field, decs, d: int):
        """Every leaf under a nest agrees with the last one on that nest's
        entries (create_struct's child-length check, StructArray::try_new),
        at every node of the tree -- not only against the first leaf."""
        n = decs[-1].counts[d]
        if any(x.counts[d] != n for x in decs):
            raise N.StrawboatError(N.E_OUT_OF_SPEC, "leaf columns of one field disagree on their rows")
        if f.kind == "struct":
            k = 0
            for c in f.children:
                m = c.n_columns()
                self._check_counts(c, decs[k:k + m], d + 1)
                k += m
        elif f.kind != "leaf":
            self._check_counts(f.children[0], decs, d + 1)

    def decode(self) -> DeviceArray:
        outs = [dec.decode() for dec in self.decoders]
        return self._assemble(self.field, list(zip(self.decoders, outs)), 0)

    def _assemble(self, f: Field, leaves, d: int) -> DeviceArray:
        dec, (offs, valid, values, leafv) = leaves[-1]
        n = dec.counts[d]
        if f.kind == "leaf":
            return DeviceArray("leaf", n, leafv, values=values)
        if f.kind == "struct":
            kids, k = [], 0
            for c in f.children:
                m = c.n_columns()
                kids.append(self._assemble(c, leaves[k:k + m], d + 1))
                k += m
            return DeviceArray("struct", n, valid[d], children=kids)
        return DeviceArray(f.kind, n, valid[d], offsets=offs[d], children=[self._assemble(f.children[0], leaves, d + 1)])

    def close(self):
        for dec in getattr(self, "decoders", []):
            dec.close()
        self.decoders = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- the writer half: any nested field through sb_encode_nested_column -------
@dataclass
class HostArray:
    """A host array of a nested Field, shaped like arrow2's arrays (the
    writer's input, NativeWriter::write, write/writer.rs:113-143).
    validity: bool per slot or None; list / large_list / map: offsets (int64,
    length + 1, absolute positions into children[0]); struct: children (each
    with one slot per struct slot); leaf: values -- fixed width: a numpy
    array; Boolean: bool per slot; Binary / Utf8: (int64 offsets, bytes)."""
    kind: str
    length: int
    validity: object = None
    offsets: object = None
    children: List["HostArray"] = field(default_factory=list)
    values: object = None


class NestInC(ctypes.Structure):
    _fields_ = [("h_offsets", ctypes.c_void_p), ("h_validity", ctypes.c_void_p)]


def _encode_lib():
    L = N.lib()
    if not getattr(L, "_nested_enc_ready", False):
        P, U64, I32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32
        L.sb_encode_nested_column.argtypes = [ctypes.POINTER(NestedDescC), ctypes.POINTER(NestInC), P, P, U64, P, U64,
                                              ctypes.POINTER(N.WriteOptionsC), U64, I32,
                                              ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(U64),
                                              ctypes.POINTER(ctypes.POINTER(N.PageMetaC)), ctypes.POINTER(U64)]
        L.sb_encode_nested_column.restype = I32
        L._nested_enc_ready = True
    return L


def _arrays_on_path(arr: HostArray, path):
    out = [arr]
    for d in range(len(path) - 1):
        f, child = path[d], path[d + 1]
        a = out[-1]
        out.append(a.children[0] if f.kind in ("list", "large_list", "map") else a.children[f.children.index(child)])
    return out


def _bits(v):
    return None if v is None else np.packbits(np.asarray(v, bool), bitorder="little")


def encode_field(fld: Field, arr: HostArray, options=None, n_threads: int = 0):
    """encode_chunk for one nested field (write/common.rs:60-115): one
    column chunk per leaf, to_leaves order, each paged by
    options.max_page_size top-level rows (slice_parquet_array) and written
    by write_nested (serialize.rs:135-198) through the host encoder
    (sb_encode_nested_column).  Returns [(chunk bytes, [PageMeta])]."""
    from .write import WriteOptions, _take

    if fld.kind == "leaf":
        raise N.StrawboatError(N.E_ARG, "a primitive field is not nested: use encode_column")
    L = _encode_lib()
    options = options or WriteOptions()
    opts = options.c()
    out_cols = []
    for path in fld.leaf_paths():
        nulls, mask, leaf_null, large = init_chain(path)
        depth = len(nulls)
        if depth > MAX_NEST:
            raise N.StrawboatError(N.E_NYI, f"nesting depth {depth} not supported")
        arrs = _arrays_on_path(arr, path)
        keep = []  # numpy buffers alive across the call
        nests = (NestInC * MAX_NEST)()
        for d in range(depth):
            a = arrs[d]
            if not (mask >> d) & 1:
                o = np.ascontiguousarray(a.offsets, np.int64)
                keep.append(o)
                nests[d].h_offsets = o.ctypes.data
            vb = _bits(a.validity)
            if vb is not None:
                keep.append(vb)
                nests[d].h_validity = vb.ctypes.data
        lf, la = path[-1], arrs[-1]
        phys = lf.physical_type
        lo = None
        vlen = 0
        if phys in (BINARY, UTF8, LARGE_BINARY, LARGE_UTF8):
            lo_, data = la.values
            lo = np.ascontiguousarray(lo_, np.int64)
            vals = np.frombuffer(data, np.uint8) if len(data) else np.zeros(1, np.uint8)
            vlen = len(data)
        elif phys == N.BOOLEAN:
            vals = _bits(la.values)
            if len(vals) == 0:
                vals = np.zeros(1, np.uint8)
        else:
            vals = np.ascontiguousarray(la.values)
            if len(vals) == 0:
                vals = np.zeros(1, vals.dtype)
        lvb = _bits(la.validity)
        ln = (ctypes.c_int32 * MAX_NEST)(*([int(x) for x in nulls] + [0] * (MAX_NEST - depth)))
        desc = NestedDescC(phys, depth, ln, int(leaf_null), 8 if large else 4, mask)
        out = ctypes.POINTER(ctypes.c_uint8)()
        olen, npg = ctypes.c_uint64(), ctypes.c_uint64()
        metas = ctypes.POINTER(N.PageMetaC)()
        vp = lambda x: None if x is None else x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        st = L.sb_encode_nested_column(ctypes.byref(desc), nests, vp(vals), vp(lo), vlen, vp(lvb), arr.length,
                                       ctypes.byref(opts), options.max_page_size or 0, n_threads, ctypes.byref(out),
                                       ctypes.byref(olen), ctypes.byref(metas), ctypes.byref(npg))
        if st:
            raise N.StrawboatError(st, "encode_nested_column")
        pm = [PageMeta(metas[i].length, metas[i].num_values) for i in range(npg.value)]
        L.sb_free(metas)
        out_cols.append((_take(out, olen.value), pm))
    return out_cols


def batch_read_field(fld: Field, columns, ctx: Optional[Context] = None) -> DeviceArray:
    """batch_read_array for a nested field (List / Map / Struct trees):
    columns = one (chunk, page metas) per leaf, to_leaves order."""
    dec = FieldDecoder(fld, columns, ctx)
    try:
        return dec.decode()
    finally:
        dec.close()
