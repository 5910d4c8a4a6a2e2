"""File side of the reader on the host (no GPU): the IPC schema parse
(infer_schema, read/reader.rs:227-241) checked leaf by leaf against
pyarrow's own type tree, and the footer read (read_meta / read_meta_async
with its 64 KiB pre-read, reader.rs:168-225) against the Python restatement
read_meta, including footers larger than the pre-read."""
import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")

import pa_amd  # noqa: E402
from pa_amd import _native as N  # noqa: E402

PHYS = {pa.int8(): N.INT8, pa.int16(): N.INT16, pa.int32(): N.INT32, pa.int64(): N.INT64, pa.uint8(): N.UINT8,
        pa.uint16(): N.UINT16, pa.uint32(): N.UINT32, pa.uint64(): N.UINT64, pa.float32(): N.FLOAT32,
        pa.float64(): N.FLOAT64, pa.bool_(): N.BOOLEAN, pa.binary(): 11, pa.large_binary(): 12, pa.utf8(): 13,
        pa.large_utf8(): 14, pa.date32(): N.INT32, pa.date64(): N.INT64, pa.timestamp("us"): N.INT64,
        pa.time32("s"): N.INT32, pa.time64("ns"): N.INT64, pa.duration("ms"): N.INT64, pa.float16(): 0,
        pa.decimal128(9, 2): 0}


def expected_leaves(schema):
    """arrow2 to_leaves order, from pyarrow's type tree, with the InitNested
    chain of each leaf (read/deserialize.rs:202-230): List / LargeList / Map
    nests and Struct nests, numbered in pre-order."""
    out = []
    nid = [0]

    def walk(f, top, nests, flags):
        t = f.type
        if pa.types.is_map(t):
            me = (f.nullable, False, "map", nid[0])
            nid[0] += 1
            walk(pa.field("entries", pa.struct([t.key_field, t.item_field]), False), top, nests + [me], flags | 2)
        elif pa.types.is_list(t) or pa.types.is_large_list(t):
            me = (f.nullable, pa.types.is_large_list(t), "list", nid[0])
            nid[0] += 1
            walk(t.value_field, top, nests + [me], flags)
        elif pa.types.is_struct(t):
            me = (f.nullable, False, "struct", nid[0])
            nid[0] += 1
            for i in range(t.num_fields):
                walk(t.field(i), top, nests + [me], flags | 1)
        else:
            sm = sum(1 << d for d, x in enumerate(nests) if x[2] == "struct")
            mm = sum(1 << d for d, x in enumerate(nests) if x[2] == "map")
            out.append((f.name, PHYS[t], f.nullable, len(nests), [x[0] for x in nests], [x[1] for x in nests], flags, top,
                        sm, mm, [x[3] for x in nests]))

    for i, f in enumerate(schema):
        walk(f, i, [], 0)
    return out


SCHEMAS = [
    pa.schema([pa.field("a", pa.int32(), False)]),
    pa.schema([pa.field(n, t, bool(i % 2)) for i, (t, n) in enumerate(
        [(pa.int8(), "i8"), (pa.uint16(), "u16"), (pa.int64(), "i64"), (pa.uint64(), "u64"), (pa.float32(), "f"),
         (pa.float64(), "d"), (pa.bool_(), "b"), (pa.utf8(), "s"), (pa.large_utf8(), "ls"), (pa.binary(), "bin"),
         (pa.large_binary(), "lbin"), (pa.date32(), "d32"), (pa.date64(), "d64"), (pa.timestamp("us"), "ts"),
         (pa.time32("s"), "t32"), (pa.time64("ns"), "t64"), (pa.duration("ms"), "dur"), (pa.float16(), "half"),
         (pa.decimal128(9, 2), "dec")])]),
    pa.schema([pa.field("l", pa.list_(pa.field("item", pa.int32(), True)), True),
               pa.field("ll", pa.list_(pa.field("x", pa.list_(pa.field("y", pa.utf8(), False)), False)), True),
               pa.field("L", pa.large_list(pa.bool_()), False)]),
    pa.schema([pa.field("st", pa.struct([pa.field("x", pa.int16()), pa.field("y", pa.list_(pa.float64()))])),
               pa.field("z", pa.uint8())]),
    pa.schema([pa.field("m", pa.map_(pa.int32(), pa.large_binary()), True),
               pa.field("lm", pa.list_(pa.field("item", pa.map_(pa.utf8(), pa.struct([pa.field("p", pa.bool_()),
                                                                                       pa.field("q", pa.int8())])),
                                                 True)), False),
               pa.field("ss", pa.struct([pa.field("a", pa.struct([pa.field("b", pa.int64(), False)]), True)]), False)]),
    pa.schema([pa.field("col_%d" % i, pa.int64()) for i in range(300)]),
]


@pytest.mark.parametrize("k", range(len(SCHEMAS)))
@pytest.mark.parametrize("framing", ["message", "encapsulated"])
def test_parse_schema_matches_pyarrow(k, framing):
    s = SCHEMAS[k]
    b = s.serialize().to_pybytes()
    if framing == "message":  # arrow2 schema_to_bytes: the Message flatbuffer alone
        b = b[8:]
    got = [(l.name, l.physical_type, l.nullable, l.depth, l.list_nullable, l.large_list, l.flags, l.top_field,
            l.struct_mask, l.map_mask, l.nest_id) for l in pa_amd.parse_schema(b)]
    assert got == expected_leaves(s)


@pytest.mark.parametrize("bad", [b"", b"\x00" * 3, b"\xff\xff\xff\xff\x08\x00\x00\x00", bytes(range(64)),
                                 b"\x10\x00\x00\x00" + b"\xff" * 60])
def test_parse_schema_rejects_garbage(bad):
    with pytest.raises(pa_amd.StrawboatError):
        pa_amd.parse_schema(bad)


def test_parse_schema_truncated_never_crashes():
    b = SCHEMAS[2].serialize().to_pybytes()[8:]
    for n in range(0, len(b), 7):
        try:
            pa_amd.parse_schema(b[:n])
        except pa_amd.StrawboatError:
            pass


def _file(tmp_path, cols, schema, name="t.sb"):
    data = pa_amd.assemble_file(cols, schema.serialize().to_pybytes()[8:])
    p = tmp_path / name
    p.write_bytes(data)
    return p, data


@pytest.mark.parametrize("page_rows", [4096, 7])  # 7 rows a page: a footer far past the 64 KiB pre-read
def test_file_open_matches_read_meta(tmp_path, page_rows):
    rng = np.random.default_rng(1)
    opts = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=page_rows)
    a = rng.integers(0, 1000, 20000).astype(np.int32)
    b = rng.random(20000)
    cols = [pa_amd.encode_column(a, None, False, opts), pa_amd.encode_column(b, rng.random(20000) > 0.3, True, opts)]
    schema = pa.schema([pa.field("a", pa.int32(), False), pa.field("b", pa.float64(), True)])
    p, data = _file(tmp_path, cols, schema)
    with pa_amd.StrawboatFile(p) as f:
        assert f.columns == pa_amd.read_meta(data)
        assert [l.name for l in f.leaves] == ["a", "b"]
        assert f.schema_bytes == schema.serialize().to_pybytes()[8:]
        for c, (chunk, pages) in enumerate(cols):
            assert f.columns[c].pages == list(pages)
            off = f.columns[c].offset
            assert data[off:off + f.columns[c].total_len()] == chunk


def test_file_open_errors(tmp_path):
    with pytest.raises(pa_amd.StrawboatError):
        pa_amd.StrawboatFile(tmp_path / "missing.sb")
    p = tmp_path / "short.sb"
    p.write_bytes(b"ARROW2\x00\x00")
    with pytest.raises(pa_amd.StrawboatError):
        pa_amd.StrawboatFile(p)
    p.write_bytes(b"ARROW2\x00\x00" + b"\x00" * 8 + (1 << 30).to_bytes(4, "little") + b"\xff" * 4 + b"\x00" * 4)
    with pytest.raises(pa_amd.StrawboatError):
        pa_amd.StrawboatFile(p)


def _fb_u32(b, p):
    return int.from_bytes(b[p:p + 4], "little")


def _fb_field(b, t, i):
    vt = t - int.from_bytes(b[t:t + 4], "little", signed=True)
    vsz = int.from_bytes(b[vt:vt + 2], "little")
    if 4 + 2 * i + 2 > vsz:
        return 0
    o = int.from_bytes(b[vt + 4 + 2 * i:vt + 6 + 2 * i], "little")
    return t + o if o else 0


def test_parse_schema_aliased_children_bounded():
    """A footer whose Struct child vectors point both entries at one table
    (2^depth visits) is rejected after a bounded walk, not walked forever
    (sb_file.cpp schema walk)."""
    t = pa.int32()
    for _ in range(40):
        t = pa.struct([pa.field("a", t), pa.field("b", pa.int32())])
    b = bytearray(pa.schema([pa.field("s", t)]).serialize().to_pybytes()[8:])
    msg = _fb_u32(b, 0)
    sch = _fb_field(b, msg, 2)
    sch += _fb_u32(b, sch)
    fv = _fb_field(b, sch, 1)
    fv += _fb_u32(b, fv)
    f = fv + 4 + _fb_u32(b, fv + 4)
    patched = 0
    while True:
        cf = _fb_field(b, f, 5)
        if not cf:
            break
        v = cf + _fb_u32(b, cf)
        if _fb_u32(b, v) != 2:
            break
        e0, e1 = v + 4, v + 8
        child0 = e0 + _fb_u32(b, e0)
        b[e1:e1 + 4] = (child0 - e1).to_bytes(4, "little")  # entry 1 aliases entry 0
        patched += 1
        f = child0
    assert patched == 40
    with pytest.raises(N.StrawboatError):
        pa_amd.parse_schema(bytes(b))


def _tree(f):
    """(kind, nullable, children | physical type) of a pa_amd.Field."""
    if f.kind == "leaf":
        return ("leaf", f.nullable, f.physical_type)
    return (f.kind, f.nullable, [_tree(c) for c in f.children])


def test_file_fields_rebuild_struct_map_trees(tmp_path):
    """StrawboatFile.field(top): the leaves' nest chains (struct / map masks,
    pre-order nest ids) regroup into each top-level field's tree -- the
    Field deserialize_nested walks (read/deserialize.rs:140-233)."""
    from tests import nestgen

    shapes = nestgen.shapes()
    names = list(shapes)
    fields = []
    for k in names:
        f = shapes[k]
        f.name = k
        fields.append(f)
    schema = pa.schema([nestgen.pa_field(f) for f in fields] + [pa.field("flat", pa.int32(), False)])
    n_leaves = sum(len(__import__("oracle.nest", fromlist=["x"]).leaf_paths(f)) for f in fields) + 1
    cols = [(b"", [])] * n_leaves
    p, _ = _file(tmp_path, cols, schema)
    with pa_amd.StrawboatFile(p) as sf:
        assert len(sf.leaves) == n_leaves
        c0 = 0
        for top, f in enumerate(fields):
            got, cols_of = sf.field(top)
            assert _tree(got) == _tree(nestgen.pa_amd_field(f)), names[top]
            k = len(cols_of)
            assert cols_of == list(range(c0, c0 + k))
            c0 += k
        got, cols_of = sf.field(len(fields))
        assert _tree(got) == ("leaf", False, N.INT32) and cols_of == [n_leaves - 1]
