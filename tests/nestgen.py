"""Nested (Struct / Map / List) columns for the tests: a random array of a
field spec (oracle.nest.F), the same array as a pyarrow array, and the
reference's integration shapes (tests/it/io.rs:167-278, 294-341) plus
nullable-struct variants.

Children of a null struct / list slot are null where they are nullable
(and lists under them empty): the arrays pyarrow builds from Python None
are not (`pa.array([None], struct)` keeps valid children), and arrow2's
level writer (RepLevelsIter / DefLevelsIter) reads the children's own
validity under a null struct, so only such arrays round-trip through the
reference writer."""
from __future__ import annotations

import numpy as np

from oracle.nest import A, F

LEAF_DTYPES = {"i32": np.int32, "i64": np.int64, "f64": np.float64, "u8": np.uint8, "i16": np.int16}


def leaf(kind, nullable, name="", large=False):
    if kind in ("utf8", "binary"):
        return F("leaf", nullable, leaf="binary", large=large, name=name)
    if kind == "bool":
        return F("leaf", nullable, leaf="bool", name=name)
    return F("leaf", nullable, leaf="fixed", dtype=np.dtype(LEAF_DTYPES[kind]), name=name)


def lst(child, nullable, name="", large=False):
    return F("large_list" if large else "list", nullable, [child], name=name)


def struct(children, nullable, name=""):
    return F("struct", nullable, list(children), name=name)


def map_(key, value, nullable, name=""):
    return F("map", nullable, [struct([key, value], False, "entries")], name=name)


def gen(f: F, n: int, rng, parent_valid=None, null_density=0.2, uniq=None) -> A:
    """A random array of field f with n slots; parent_valid (bool per slot
    or None) nulls the nullable children of null parents."""
    pv = np.ones(n, bool) if parent_valid is None else parent_valid
    validity = None
    if f.nullable:
        validity = (rng.random(n) >= null_density) & pv
    live = pv if validity is None else validity
    if f.kind == "leaf":
        if f.leaf == "fixed":
            dt = f.dtype
            hi = uniq or max(2, n)
            if dt.kind == "f":
                vals = rng.integers(0, hi, n).astype(dt)
            else:
                vals = rng.integers(0, min(hi, np.iinfo(dt).max), n).astype(dt)
            return A("leaf", n, validity, values=vals)
        if f.leaf == "bool":
            return A("leaf", n, validity, values=rng.random(n) < 0.5)
        hi = uniq or max(2, n)
        strs = [str(int(x)).encode() for x in rng.integers(0, hi, n)]
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum([len(s) for s in strs])
        return A("leaf", n, validity, values=(offs, b"".join(strs)))
    if f.kind == "struct":
        kids = [gen(c, n, rng, live, null_density, uniq) for c in f.children]
        return A("struct", n, validity, children=kids)
    # list / map: lengths uniform {0, 1, 2} (io.rs:399-415), null / dead slots empty
    lens = np.where(live, rng.integers(0, 3, n), 0)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    child = gen(f.children[0], int(offs[-1]), rng, None, null_density, uniq)
    return A(f.kind, n, validity, offsets=offs, children=[child])


def pa_type(f: F):
    import pyarrow as pa

    if f.kind == "leaf":
        if f.leaf == "binary":
            return pa.large_binary() if f.large else pa.binary()
        if f.leaf == "bool":
            return pa.bool_()
        return pa.from_numpy_dtype(f.dtype)
    if f.kind == "struct":
        return pa.struct([pa_field(c) for c in f.children])
    if f.kind == "map":
        e = f.children[0]
        return pa.map_(pa_field(e.children[0]), pa_field(e.children[1]))
    t = pa_field(f.children[0])
    return pa.large_list(t) if f.kind == "large_list" else pa.list_(t)


def pa_field(f: F):
    import pyarrow as pa

    return pa.field(f.name or "item", pa_type(f), nullable=f.nullable)


def to_pa(f: F, a: A):
    """The same array in pyarrow (children as they are, nulls and all)."""
    import pyarrow as pa

    mask = None if a.validity is None else pa.array(~np.asarray(a.validity, bool))
    if f.kind == "leaf":
        if f.leaf == "binary":
            offs, data = a.values
            vals = [None if (a.validity is not None and not a.validity[i]) else data[offs[i]:offs[i + 1]]
                    for i in range(a.length)]
            return pa.array(vals, type=pa_type(f))
        return pa.array(a.values, type=pa_type(f), mask=None if a.validity is None else ~np.asarray(a.validity, bool))
    if f.kind == "struct":
        kids = [to_pa(c, x) for c, x in zip(f.children, a.children)]
        return pa.StructArray.from_arrays(kids, fields=[pa_field(c) for c in f.children], mask=mask)
    if f.kind == "map":
        e, ea = f.children[0], a.children[0]
        keys, items = to_pa(e.children[0], ea.children[0]), to_pa(e.children[1], ea.children[1])
        return pa.MapArray.from_arrays(pa.array(a.offsets.astype(np.int32)), keys, items, type=pa_type(f),
                                       mask=mask)
    child = to_pa(f.children[0], a.children[0])
    if f.kind == "large_list":
        return pa.LargeListArray.from_arrays(pa.array(a.offsets), child, type=pa_type(f), mask=mask)
    return pa.ListArray.from_arrays(pa.array(a.offsets.astype(np.int32)), child, type=pa_type(f), mask=mask)


def shapes():
    """name -> field: the reference's test_struct / test_map /
    test_list_struct / test_list_map / test_struct_list (io.rs:167-278) and
    variants with null structs, structs in structs, Boolean and Float leaves."""
    name_age = lambda n: struct([leaf("binary", True, "name", large=True), leaf("i32", True, "age")], n)  # noqa: E731
    kv = lambda n: map_(leaf("i32", False, "key"), leaf("binary", True, "value", large=True), n)  # noqa: E731
    return {
        "struct": name_age(False),  # io.rs:168-172, create_struct: validity None
        "map": kv(True),  # io.rs:189-193, create_map: offsets with nulls
        "list_struct": lst(name_age(True), False),  # io.rs:216-233
        "list_map": lst(kv(True), False),  # io.rs:236-253
        "struct_list": struct([leaf("binary", True, "name", large=True),
                               lst(leaf("i32", True), True, "age")], False),  # io.rs:256-278
        "null_struct": name_age(True),
        "struct_struct": struct([leaf("i64", True, "a"),
                                 struct([leaf("bool", True, "b"), leaf("f64", False, "c")], True, "s")], True),
        "list_null_struct_list": lst(struct([lst(leaf("i16", True), True, "l"), leaf("utf8", True, "u")], True), True),
        "map_of_list": map_(leaf("i32", False, "key"), lst(leaf("i64", True), True, "value"), True),
        "req_struct_req": struct([leaf("i32", False, "x"), leaf("u8", False, "y")], False),
    }


def pa_amd_field(f: F):
    """oracle.nest.F -> pa_amd.Field."""
    import pa_amd
    from pa_amd import _native as N

    if f.kind == "leaf":
        if f.leaf == "binary":
            return pa_amd.Field.leaf(pa_amd.LARGE_BINARY if f.large else pa_amd.BINARY, f.nullable, f.name)
        if f.leaf == "bool":
            return pa_amd.Field.leaf(N.BOOLEAN, f.nullable, f.name)
        return pa_amd.Field.leaf(f.dtype, f.nullable, f.name)
    return pa_amd.Field(f.kind, f.nullable, [pa_amd_field(c) for c in f.children], name=f.name)


def device_to_host(f: F, d) -> A:
    """pa_amd.DeviceArray -> oracle.nest.A (bitmaps unpacked)."""
    n = d.length

    def bits(t, k):
        return np.unpackbits(t.cpu().numpy().view(np.uint8), bitorder="little")[:k].astype(bool)

    validity = None if d.validity is None else bits(d.validity, n)
    if f.kind == "leaf":
        if f.leaf == "fixed":
            v = d.values.cpu().numpy().view(np.uint8)[: n * f.dtype.itemsize].view(f.dtype)
        elif f.leaf == "bool":
            v = bits(d.values, n)
        else:
            o = d.values[0].cpu().numpy().astype(np.int64)[: n + 1]
            v = (o, d.values[1].cpu().numpy().tobytes()[: int(o[-1]) if n else 0])
        return A("leaf", n, validity, values=v)
    if f.kind == "struct":
        return A("struct", n, validity, children=[device_to_host(c, x) for c, x in zip(f.children, d.children)])
    offs = d.offsets.cpu().numpy().astype(np.int64)[: n + 1]
    return A(f.kind, n, validity, offsets=offs, children=[device_to_host(f.children[0], d.children[0])])


# ---- the reference's integration chunks as io.rs builds them ---------------
def _rand_index(n, null_density, uniq, rng, dtype=np.int32):
    """create_random_index (io.rs:357-369): Some(v in [0, uniq)) or None (0)."""
    valid = rng.random(n) > null_density
    v = np.where(valid, rng.integers(0, max(uniq, 1), n), 0).astype(dtype)
    return A("leaf", n, valid, values=v)


def _rand_string(n, null_density, uniq, rng):
    """create_random_string (io.rs:385-397): decimal strings or None (empty)."""
    valid = rng.random(n) > null_density
    vals = rng.integers(0, max(uniq, 1), n)
    strs = [str(int(x)).encode() if ok else b"" for x, ok in zip(vals, valid)]
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum([len(s) for s in strs])
    return A("leaf", n, valid, values=(offs, b"".join(strs)))


def _rand_bool(n, null_density, rng):
    valid = rng.random(n) > null_density
    return A("leaf", n, valid, values=(rng.random(n) < 0.5) & valid)


def _rand_offsets(n, null_density, rng):
    """create_random_offsets (io.rs:399-415): lengths {0, 1, 2}, null lists empty."""
    valid = rng.random(n) > null_density
    lens = np.where(valid, rng.integers(0, 3, n), 0)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    return offs, valid


def _create_list(n, null_density, rng, item=None):
    offs, valid = _rand_offsets(n, 0.1, rng)
    m = int(offs[-1])
    child = item(m) if item else _rand_index(m, null_density, m, rng)
    return A("list", n, valid, offsets=offs, children=[child])


def _create_struct(n, null_density, uniq, rng):
    return A("struct", n, None, children=[_rand_string(n, null_density, uniq, rng),
                                          _rand_index(n, null_density, uniq, rng)])


def _create_map(n, null_density, rng):
    offs, valid = _rand_offsets(n, 0.1, rng)
    m = int(offs[-1])
    entries = A("struct", m, None, children=[_rand_index(m, 0.0, m, rng), _rand_string(m, null_density, m, rng)])
    return A("map", n, valid, offsets=offs, children=[entries])


def _stride2(child, rows=500):
    """io.rs:199-205: ListArray over offsets 0, 2, .., 2 * rows of a longer child."""
    return A("list", rows, None, offsets=np.arange(0, 2 * rows + 1, 2, dtype=np.int64), children=[child])


def io_rs_cases(rng):
    """name -> (field, array): test_struct, test_map, test_list_list,
    test_list_struct, test_list_map, test_struct_list (io.rs:167-278) as
    test_write_read_with_options declares them (top field nullable iff the
    array has a validity, :444-452), plus List<Utf8>, List<Boolean> and
    List<List<Boolean>> leaves."""
    name_age = struct([leaf("binary", True, "name", large=True), leaf("i32", True, "age")], False)
    name_age_item = struct([leaf("binary", True, "name", large=True), leaf("i32", True, "age")], True, "item")
    kv = lambda n: map_(leaf("i32", False, "key"), leaf("binary", True, "value", large=True), n)  # noqa: E731
    int_list = lambda n, name="": lst(leaf("i32", True, "item"), n, name)  # noqa: E731
    cases = {
        "test_struct": (name_age, _create_struct(1000, 0.2, 1000, rng)),
        "test_map": (kv(True), _create_map(1000, 0.2, rng)),
        "test_list_list": (lst(int_list(True, "item"), False), _stride2(_create_list(2000, 0.2, rng))),
        "test_list_struct": (lst(name_age_item, False), _stride2(_create_struct(2000, 0.2, 2000, rng))),
        "test_list_map": (lst(kv(True), False), _stride2(_create_map(2000, 0.2, rng))),
        "test_struct_list": (struct([leaf("binary", True, "name", large=True), int_list(True, "age")], False),
                             A("struct", 10000, None, children=[_rand_string(10000, 0.2, 10000, rng),
                                                               _create_list(10000, 0.2, rng)])),
        "list_utf8": (lst(leaf("utf8", True, "item"), True),
                      _create_list(3000, 0.2, rng, lambda m: _rand_string(m, 0.2, 50, rng))),
        "list_bool": (lst(leaf("bool", True, "item"), True),
                      _create_list(3000, 0.2, rng, lambda m: _rand_bool(m, 0.2, rng))),
        "list_list_bool": (lst(lst(leaf("bool", False, "item"), True, "item"), True),
                           _create_list(1500, 0.2, rng, lambda m: _create_list(
                               m, 0.2, rng, lambda k: A("leaf", k, None, values=rng.random(k) < 0.3)))),
    }
    return cases


def host_array(a: A):
    """oracle.nest.A -> pa_amd.HostArray (the product writer's input)."""
    import pa_amd

    return pa_amd.HostArray(a.kind, a.length, a.validity, a.offsets, [host_array(c) for c in a.children], a.values)


def _slice(a: A, b: int, e: int) -> A:
    """Slots [b, e) of an array (children compacted to the slots they reach)."""
    v = None if a.validity is None else np.asarray(a.validity)[b:e]
    if a.kind == "leaf":
        if isinstance(a.values, tuple):
            offs, data = a.values
            o = np.asarray(offs[b:e + 1], np.int64)
            return A("leaf", e - b, v, values=(o - o[0], data[int(o[0]):int(o[-1])]))
        return A("leaf", e - b, v, values=np.asarray(a.values)[b:e])
    if a.kind == "struct":
        return A("struct", e - b, v, children=[_slice(c, b, e) for c in a.children])
    o = np.asarray(a.offsets[b:e + 1], np.int64)
    return A(a.kind, e - b, v, offsets=o - o[0], children=[_slice(a.children[0], int(o[0]), int(o[-1]))])


def compact(a: A) -> A:
    """The array with every child cut to the slots its parent reaches (what
    Arrow logical equality compares, e.g. io.rs's ListArray over the first
    half of a longer child)."""
    return _slice(a, 0, a.length)
