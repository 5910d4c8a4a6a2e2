"""Struct / Map / List nesting for the oracle (TEST INFRASTRUCTURE ONLY: only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it).

A nested field (List / LargeList / Map / Struct over primitive, Boolean and
Binary / Utf8 leaves) is written as one column chunk per leaf, in to_leaves
order, and read back leaf by leaf -- the reference's shape:

  writer  encode_chunk  write/common.rs:49-119 (to_nested, to_leaves, pages
          of max_page_size top-level rows, PageMeta.num_values = the page's
          level count, arrow2 num_values)
          write_nested / write_nested_validity  write/serialize.rs:133-146,
          217-232 (arrow2 write_rep_and_def V2: no stream when the max level
          is 0; parquet2 encode_u32 otherwise)
  reader  deserialize_nested  read/deserialize.rs:140-233 (InitNested chain:
          List / Map push InitNested::List, Struct pushes InitNested::Struct
          once per child), read_validity_nested read/read_basic.rs:65-173
          (orc_read_nest_page), create_list / create_map (read/array/list.rs,
          map.rs), create_struct (read/array/struct_.rs:101-114: the struct's
          validity is the LAST child's), batch_read.rs:128-180 (the same for
          whole columns).

The levels are restated as the Dremel encoding arrow2's RepLevelsIter /
DefLevelsIter produce for arrays whose children are null under a null
parent (the arrays arrow2 / pyarrow build from Python None); they are pinned
against pyarrow's parquet writer (tests/test_pyarrow_nested.py)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import oracle as O

LEAF_KINDS = ("fixed", "binary", "bool")


@dataclass
class F:
    """An arrow2 Field restricted to the codec path.  kind: "list",
    "large_list", "map", "struct" or "leaf"; a map's single child is its
    entries struct (key, value); a leaf has `leaf` in LEAF_KINDS and a dtype
    (fixed width), `large` offsets (binary)."""
    kind: str
    nullable: bool
    children: List["F"] = field(default_factory=list)
    leaf: str = "fixed"
    dtype: object = None
    large: bool = False
    name: str = ""


@dataclass
class A:
    """A host array of field F.  validity: bool per slot or None;
    list / map: offsets (int64, len + 1) and children[0]; struct: children;
    leaf fixed: values; bool: values (bool); binary: values = (int64
    offsets, bytes)."""
    kind: str
    length: int
    validity: Optional[np.ndarray] = None
    offsets: Optional[np.ndarray] = None
    children: List["A"] = field(default_factory=list)
    values: object = None


def n_columns(f: F) -> int:
    """arrow2 n_columns: leaves under f."""
    return 1 if f.kind == "leaf" else sum(n_columns(c) for c in f.children)


def leaf_paths(f: F, prefix=()):
    """to_leaves order: depth first, children in order -> tuples of fields
    from the top field to the leaf."""
    path = prefix + (f,)
    if f.kind == "leaf":
        return [path]
    out = []
    for c in f.children:
        out += leaf_paths(c, path)
    return out


def init_chain(path):
    """The InitNested chain of deserialize_nested for one leaf path ->
    (nest nullable per nest, struct_mask, leaf nullable).  A list / map nest
    is InitNested::List(field nullable); a struct nest InitNested::Struct
    (the struct field's nullable, deserialize.rs:215-226)."""
    nulls, mask = [], 0
    for d, f in enumerate(path[:-1]):
        nulls.append(bool(f.nullable))
        if f.kind == "struct":
            mask |= 1 << d
    return tuple(nulls), mask, bool(path[-1].nullable)


def _max_levels(path):
    nulls, mask, leaf_null = init_chain(path)
    max_rep = sum(0 if (mask >> d) & 1 else 1 for d in range(len(nulls)))
    max_def = sum(int(n) + (0 if (mask >> d) & 1 else 1) for d, n in enumerate(nulls)) + int(leaf_null)
    return max_rep, max_def


def _arrays_on_path(arr: A, path):
    """The arrays along a leaf path (the top array, then the child on the path)."""
    out = [arr]
    for d in range(len(path) - 1):
        f, child = path[d], path[d + 1]
        a = out[-1]
        out.append(a.children[0] if f.kind in ("list", "large_list", "map") else a.children[f.children.index(child)])
    return out


def levels(arr: A, path, r0: int, r1: int):
    """Dremel rep / def levels of rows [r0, r1) of the leaf at `path`, and
    the leaf slot range [j0, j1) those rows cover (slice_parquet_array).  A
    null or empty list emits one level; a struct passes through (every child
    of a struct slot, null or not, is one leaf slot of the leaf array); the
    leaf adds its own validity."""
    arrs = _arrays_on_path(arr, path)
    D = len(path) - 1
    cum_rep = [0] * (D + 2)
    for d, f in enumerate(path):
        cum_rep[d + 1] = cum_rep[d] + (1 if f.kind in ("list", "large_list", "map") else 0)
    reps, defs = [], []

    def valid(a, i):
        return a.validity is None or bool(a.validity[i])

    def walk(d, i, rep, dl):
        f, a = path[d], arrs[d]
        if d == D:
            reps.append(rep)
            defs.append(dl + int(f.nullable and valid(a, i)))
            return
        if f.nullable and not valid(a, i):
            reps.append(rep)
            defs.append(dl)
            return
        dl += int(f.nullable)
        if f.kind == "struct":
            walk(d + 1, i, rep, dl)
            return
        b, e = int(a.offsets[i]), int(a.offsets[i + 1])
        if b == e:
            reps.append(rep)
            defs.append(dl)
            return
        for k, j in enumerate(range(b, e)):
            walk(d + 1, j, rep if k == 0 else cum_rep[d + 1], dl + 1)

    for i in range(r0, r1):
        walk(0, i, 0, 0)
    # leaf slot range: map the rows through each list nest's offsets
    j0, j1 = r0, r1
    for d in range(D):
        if path[d].kind != "struct":
            o = arrs[d].offsets
            j0, j1 = int(o[j0]), int(o[j1])
    return np.asarray(reps, np.uint32), np.asarray(defs, np.uint32), j0, j1


def _levels_page(rep, dfl, max_rep, max_def, rows):
    L = O.lib()
    if not getattr(L, "_lvpage_ready", False):
        import ctypes

        L.orc_write_levels_page.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(O._Buf)]
        L._lvpage_ready = True
    import ctypes

    buf = O._Buf()
    r = np.ascontiguousarray(rep, np.uint32) if len(rep) else np.zeros(1, np.uint32)
    d = np.ascontiguousarray(dfl, np.uint32) if len(dfl) else np.zeros(1, np.uint32)
    rc = L.orc_write_levels_page(O._ptr(r), O._ptr(d), len(rep), max_rep, max_def, rows, ctypes.byref(buf))
    data = O._take(buf)
    O._check(rc, "write_levels_page")
    return data


def compress_binary(values: bytes, offsets, validity, opts, offset_width=4, parent_values_len=None) -> bytes:
    """compress_binary (compression/binary/mod.rs:26-93) of one leaf slice."""
    import ctypes

    L = O._bin_lib()
    if not getattr(L, "_cbin_ready", False):
        P = ctypes.c_void_p
        L.orc_compress_binary.argtypes = [P, P, P, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.POINTER(O.WriteOptions), ctypes.POINTER(O._Buf)]
        L._cbin_ready = True
    n = len(offsets) - 1
    offs = np.ascontiguousarray(offsets, np.int64)
    vals = np.frombuffer(values, np.uint8) if values else np.zeros(1, np.uint8)
    vb = None if validity is None else np.packbits(np.asarray(validity, bool), bitorder="little")
    buf = O._Buf()
    pl = len(values) if parent_values_len is None else parent_values_len
    rc = L.orc_compress_binary(O._ptr(vals), O._ptr(offs), O._ptr(vb), n, offset_width, pl, ctypes.byref(opts),
                               ctypes.byref(buf))
    data = O._take(buf)
    O._check(rc, "compress_binary")
    return data


def compress_bool(bits: np.ndarray, off: int, n: int, validity, opts) -> bytes:
    """compress_boolean (compression/boolean/mod.rs:23-61) of the leaf slice
    [off, off + n) of the bitmap `bits`: the Basic codecs take the parent's
    bytes when off % 8 == 0 (Bitmap::as_slice), a rebuilt bitmap otherwise."""
    import ctypes

    L = O.lib()
    if not getattr(L, "_cbool_ready", False):
        P = ctypes.c_void_p
        L.orc_compress_boolean.argtypes = [P, ctypes.c_size_t, P, ctypes.c_size_t, ctypes.POINTER(O.WriteOptions),
                                           ctypes.POINTER(O._Buf)]
        L._cbool_ready = True
    if len(bits) == 0:
        bits = np.zeros(1, np.uint8)
    vb = None if validity is None else O._pack(validity)
    buf = O._Buf()
    rc = L.orc_compress_boolean(O._ptr(bits), off, O._ptr(vb), n, ctypes.byref(opts), ctypes.byref(buf))
    data = O._take(buf)
    O._check(rc, "compress_boolean")
    return data


def leaf_stream(leaf_f: F, leaf_a: A, j0: int, j1: int, opts) -> bytes:
    """The leaf's values section of a nested page (write_nested's
    write_primitive / write_bitmap / write_binary over the sliced leaf)."""
    val = None if leaf_a.validity is None else np.asarray(leaf_a.validity[j0:j1], bool)
    if leaf_f.leaf == "fixed":
        return O.compress(np.ascontiguousarray(leaf_a.values[j0:j1]), val, opts)
    if leaf_f.leaf == "bool":  # write_bitmap over the sliced leaf: the leaf's bitmap at bit offset j0
        return compress_bool(O._pack(np.asarray(leaf_a.values, bool)), j0, j1 - j0, val, opts)
    offs, data = leaf_a.values
    b, e = int(offs[j0]), int(offs[j1])
    return compress_binary(data[b:e], np.asarray(offs[j0:j1 + 1], np.int64) - b, val, opts,
                           8 if leaf_f.large else 4, parent_values_len=len(data))


def write_field(f: F, arr: A, page_rows: int, opts=None, page_seed=None):
    """encode_chunk for one nested field -> one (chunk, [(length,
    num_levels)]) per leaf, to_leaves order.  page_seed(p), when given, is
    the sampler seed of page p (the product writer's sb_page_seed(opts.seed,
    p)); otherwise every page samples with opts.seed."""
    opts = opts or O.WriteOptions.make()
    rows = arr.length
    step = min(page_rows or rows, rows) if rows else 1
    out = []
    for path in leaf_paths(f):
        max_rep, max_def = _max_levels(path)
        leaf_a = _arrays_on_path(arr, path)[-1]
        chunk, metas = [], []
        for p, r0 in enumerate(range(0, rows, step)):
            r1 = min(rows, r0 + step)
            po = opts
            if page_seed is not None:
                po = O.WriteOptions(opts.default_codec, opts.has_ratio, opts.ratio, opts.forbidden_mask,
                                    opts.forced_codec, page_seed(p))
            rep, dfl, j0, j1 = levels(arr, path, r0, r1)
            page = _levels_page(rep, dfl, max_rep, max_def, r1 - r0) + leaf_stream(path[-1], leaf_a, j0, j1, po)
            chunk.append(page)
            metas.append((len(page), len(rep)))
        out.append((b"".join(chunk), metas))
    return out


def read_leaf(path, chunk, metas):
    """One leaf column of a nested field through orc_read_nest_page."""
    nulls, mask, leaf_null = init_chain(path)
    lf = path[-1]
    dtype = lf.dtype if lf.leaf == "fixed" else np.uint8
    offs, bits, values, leafv, counts = O.read_nested_column(
        chunk, metas, dtype, nulls, leaf_null, leaf=lf.leaf, offset_width=8 if lf.large else 4, struct_mask=mask,
        with_counts=True)
    return dict(offsets=offs, validity=bits, values=values, leaf_validity=leafv, counts=counts)


def assemble(f: F, leaves: list, d: int = 0) -> A:
    """Arrays from per-leaf reads (each a read_leaf dict, to_leaves order):
    a nest's arrays come from the LAST leaf under it -- create_list /
    create_map / create_struct pop the last child's NestedState
    (read/array/struct_.rs:101-114)."""
    last = leaves[-1]
    if f.kind == "leaf":
        assert len(leaves) == 1
        return A("leaf", last["counts"][d], last["leaf_validity"], values=last["values"])
    n = last["counts"][d]
    if f.kind == "struct":
        kids, k = [], 0
        for c in f.children:
            m = n_columns(c)
            kids.append(assemble(c, leaves[k:k + m], d + 1))
            k += m
        return A("struct", n, last["validity"][d], children=kids)
    return A(f.kind, n, last["validity"][d], offsets=last["offsets"][d], children=[assemble(f.children[0], leaves, d + 1)])


def read_field(f: F, columns) -> A:
    """batch_read_array / column_iter_to_arrays + concatenate for a nested
    field: columns = one (chunk, metas) per leaf, to_leaves order."""
    paths = leaf_paths(f)
    assert len(paths) == len(columns)
    return assemble(f, [read_leaf(p, c, m) for p, (c, m) in zip(paths, columns)])


def equal(f: F, a: A, b: A, values_under_nulls=True, path="") -> None:
    """Asserts two arrays of field f are the same: lengths, offsets,
    validity (None == all valid), and values (bit-exact, including the slots
    under nulls unless values_under_nulls is False)."""
    assert a.length == b.length, f"{path}: length {a.length} != {b.length}"

    def vmask(x):
        return np.ones(x.length, bool) if x.validity is None else np.asarray(x.validity[:x.length], bool)

    va, vb = vmask(a), vmask(b)
    assert (va == vb).all(), f"{path}: validity differs"
    if f.kind in ("list", "large_list", "map"):
        assert (np.asarray(a.offsets, np.int64) == np.asarray(b.offsets, np.int64)).all(), f"{path}: offsets differ"
        equal(f.children[0], a.children[0], b.children[0], values_under_nulls, path + "/item")
    elif f.kind == "struct":
        for c, x, y in zip(f.children, a.children, b.children):
            equal(c, x, y, values_under_nulls, path + "/" + c.name)
    else:
        keep = np.ones(a.length, bool) if values_under_nulls else va
        if f.leaf == "binary":
            (oa, da), (ob, db) = a.values, b.values
            for i in np.flatnonzero(keep):
                assert da[oa[i]:oa[i + 1]] == db[ob[i]:ob[i + 1]], f"{path}: row {i} differs"
        else:
            xa, xb = np.asarray(a.values)[:a.length], np.asarray(b.values)[:b.length]
            assert (xa[keep].view(np.uint8) if xa.dtype == bool else xa[keep]).tobytes() == \
                   (xb[keep].view(np.uint8) if xb.dtype == bool else xb[keep]).tobytes(), f"{path}: values differ"
