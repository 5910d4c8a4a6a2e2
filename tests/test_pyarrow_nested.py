"""The nested-level oracle against pyarrow (arrow2/parquet2
row).  pyarrow.parquet writes List<Int32> columns as Data Page V2 pages (rep
and def levels as RLE / bit-packed hybrid streams with explicit lengths --
the same streams a strawboat nested page carries, read_basic.rs:65-99).  Each
page's level bytes are cut out of the file (a minimal Thrift compact reader
for PageHeader), wrapped into a strawboat nested page ([rows][rep_len]
[def_len][rep][def][values], values = every leaf slot), and read back by the
oracle (orc_hybrid_decode + the read_validity_nested / create_list
restatement); offsets, list validity, values and leaf validity must equal
pyarrow's ListArray.  Runs on CPU; covers list/item nullability, empty and
null lists, several pages per column."""
import io

import numpy as np
import pytest

from oracle import oracle as O

pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")


class Compact:
    """Just enough of Thrift's compact protocol to walk a PageHeader."""

    def __init__(self, b, p):
        self.b, self.p = b, p

    def varint(self):
        v = s = 0
        while True:
            c = self.b[self.p]
            self.p += 1
            v |= (c & 0x7F) << s
            if not c & 0x80:
                return v
            s += 7

    def zz(self):
        v = self.varint()
        return (v >> 1) ^ -(v & 1)

    def value(self, t):
        if t in (1, 2):
            return t == 1
        if t == 3:
            self.p += 1
            return self.b[self.p - 1]
        if t in (4, 5, 6):
            return self.zz()
        if t == 7:
            self.p += 8
            return None
        if t == 8:
            n = self.varint()
            self.p += n
            return None
        if t in (9, 10):
            h = self.b[self.p]
            self.p += 1
            n, et = h >> 4, h & 15
            if n == 15:
                n = self.varint()
            return [self.value(et) for _ in range(n)]
        if t == 12:
            return self.struct()
        raise ValueError(f"thrift type {t}")

    def struct(self):
        out, fid = {}, 0
        while True:
            h = self.b[self.p]
            self.p += 1
            if h == 0:
                return out
            d, t = h >> 4, h & 15
            fid = fid + d if d else self.zz()
            out[fid] = self.value(t)


def data_pages_v2(path, with_encoding=False):
    """(rows, levels, rep bytes, def bytes, values bytes[, values encoding]) of each data page of column 0."""
    f = pq.ParquetFile(path)
    cm = f.metadata.row_group(0).column(0)
    raw = open(path, "rb").read()
    p, end = cm.data_page_offset, cm.data_page_offset + cm.total_compressed_size
    pages = []
    while p < end:
        c = Compact(raw, p)
        h = c.struct()
        body = raw[c.p:c.p + h[3]]
        p = c.p + h[3]
        if h[1] != 3:  # DATA_PAGE_V2 only (no dictionary pages are written)
            continue
        v2 = h[8]
        dl, rl = v2[5], v2[6]
        pg = (v2[3], v2[1], body[:rl], body[rl:rl + dl], body[rl + dl:])
        pages.append(pg + (v2[4],) if with_encoding else pg)
    return pages


def list_column(rng, rows, list_nullable, item_nullable):
    vals = []
    for _ in range(rows):
        r = rng.random()
        if list_nullable and r < 0.1:
            vals.append(None)
        elif r < 0.2:
            vals.append([])
        else:
            vals.append([None if item_nullable and rng.random() < 0.15 else int(x)
                         for x in rng.integers(-1000, 1000, int(rng.integers(1, 7)))])
    field = pa.field("c", pa.list_(pa.field("item", pa.int32(), nullable=item_nullable)), nullable=list_nullable)
    return pa.table({"c": pa.array(vals, type=field.type)}, schema=pa.schema([field]))


@pytest.mark.parametrize("list_nullable", [False, True], ids=["list_req", "list_null"])
@pytest.mark.parametrize("item_nullable", [False, True], ids=["item_req", "item_null"])
def test_levels_match_pyarrow(tmp_path, list_nullable, item_nullable):
    rng = np.random.default_rng(7 + 2 * list_nullable + item_nullable)
    t = list_column(rng, 20000, list_nullable, item_nullable)
    path = str(tmp_path / "l.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False,
                   data_page_size=8192, write_statistics=False)
    pages = data_pages_v2(path)
    assert len(pages) > 3
    max_def = int(list_nullable) + 1 + int(item_nullable)
    bw = max_def.bit_length()
    chunk, metas = b"", []
    for rows, nlev, rep, dfb, plain in pages:
        d = O.hybrid_decode(dfb, bw, nlev) if dfb else np.full(nlev, max_def, np.uint32)
        # every leaf slot (def >= the leaf level) carries a value: the page's
        # PLAIN values at the non-null slots, 0 at the null ones
        slot_def = d[d >= int(list_nullable) + 1]
        page_vals = np.zeros(len(slot_def), np.int32)
        nn = slot_def == max_def
        page_vals[nn] = np.frombuffer(plain, np.int32, int(nn.sum()))
        stream = O.compress(page_vals, None, O.WriteOptions.make())
        body = rows.to_bytes(4, "little") + len(rep).to_bytes(4, "little") + len(dfb).to_bytes(4, "little")
        chunk += body + rep + dfb + stream
        metas.append((len(body) + len(rep) + len(dfb) + len(stream), nlev))
    offs, lv, vals, fv = O.read_list_column(chunk, metas, np.int32, list_nullable, item_nullable)
    (go,), (gb,), gv, gf = O.read_nested_column(chunk, metas, np.int32, (list_nullable,), item_nullable)
    assert (go == offs).all() and (gv == vals).all()  # the general reader at depth 1
    assert (gb is None) == (lv is None) and (gb is None or (gb == lv).all())
    assert (gf is None) == (fv is None) and (gf is None or (gf == fv).all())
    arr = t.column("c").combine_chunks()
    assert (offs == arr.offsets.to_numpy()).all()
    if list_nullable:
        assert (lv == arr.is_valid().to_numpy(zero_copy_only=False)).all()
    assert len(vals) == len(arr.values)
    present = arr.values.is_valid().to_numpy(zero_copy_only=False)
    assert (vals[present] == arr.values.to_numpy(zero_copy_only=False)[present]).all()
    if item_nullable:
        assert (fv == arr.values.is_valid().to_numpy(zero_copy_only=False)).all()


def list2_column(rng, rows, n0, n1, ni):
    def inner():
        r = rng.random()
        if n1 and r < 0.1:
            return None
        if r < 0.2:
            return []
        return [None if ni and rng.random() < 0.15 else int(x) for x in rng.integers(-1000, 1000, int(rng.integers(1, 5)))]

    vals = []
    for _ in range(rows):
        r = rng.random()
        if n0 and r < 0.1:
            vals.append(None)
        elif r < 0.2:
            vals.append([])
        else:
            vals.append([inner() for _ in range(int(rng.integers(1, 4)))])
    leaf = pa.field("item", pa.int32(), nullable=ni)
    mid = pa.field("item", pa.list_(leaf), nullable=n1)
    field = pa.field("c", pa.list_(mid), nullable=n0)
    return pa.table({"c": pa.array(vals, type=field.type)}, schema=pa.schema([field]))


@pytest.mark.parametrize("n0", [False, True], ids=["outer_req", "outer_null"])
@pytest.mark.parametrize("n1", [False, True], ids=["inner_req", "inner_null"])
@pytest.mark.parametrize("ni", [False, True], ids=["item_req", "item_null"])
def test_list_of_lists_match_pyarrow(tmp_path, n0, n1, ni):
    """List<List<Int32>>: the general nested reader (orc_read_nested_page,
    cum_sum / cum_rep over three nests) against pyarrow's arrays."""
    rng = np.random.default_rng(11 + 4 * n0 + 2 * n1 + ni)
    t = list2_column(rng, 8000, n0, n1, ni)
    path = str(tmp_path / "ll.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False,
                   data_page_size=4096, write_statistics=False)
    pages = data_pages_v2(path)
    assert len(pages) > 3
    leaf_def = int(n0) + 1 + int(n1) + 1
    max_def = leaf_def + int(ni)
    chunk, metas = pages_to_chunk(pages, max_def, leaf_def)
    (o0, o1), (b0, b1), vals, fv = O.read_nested_column(chunk, metas, np.int32, (n0, n1), ni)
    arr = t.column("c").combine_chunks()
    inner = arr.values
    assert (o0 == arr.offsets.to_numpy()).all()
    assert (o1 == inner.offsets.to_numpy()).all()
    if n0:
        assert (b0 == arr.is_valid().to_numpy(zero_copy_only=False)).all()
    if n1:
        assert (b1 == inner.is_valid().to_numpy(zero_copy_only=False)).all()
    leaf = inner.values
    assert len(vals) == len(leaf)
    present = leaf.is_valid().to_numpy(zero_copy_only=False)
    assert (vals[present] == leaf.to_numpy(zero_copy_only=False)[present]).all()
    if ni:
        assert (fv == present).all()


def pages_to_chunk(pages, max_def, leaf_def):
    """strawboat nested pages from pyarrow V2 data pages: levels as they are,
    values = every leaf slot (def >= leaf_def), PLAIN values at the non-null ones."""
    bw = max_def.bit_length()
    chunk, metas = b"", []
    for rows, nlev, rep, dfb, plain in pages:
        d = O.hybrid_decode(dfb, bw, nlev) if dfb else np.full(nlev, max_def, np.uint32)
        slot_def = d[d >= leaf_def]
        page_vals = np.zeros(len(slot_def), np.int32)
        nn = slot_def == max_def
        page_vals[nn] = np.frombuffer(plain, np.int32, int(nn.sum()))
        stream = O.compress(page_vals, None, O.WriteOptions.make())
        body = rows.to_bytes(4, "little") + len(rep).to_bytes(4, "little") + len(dfb).to_bytes(4, "little")
        chunk += body + rep + dfb + stream
        metas.append((len(body) + len(rep) + len(dfb) + len(stream), nlev))
    return chunk, metas


def leaf_pages(pages, max_def, leaf_def, encode):
    """strawboat nested pages whose values section is encode(slot_def, plain, encoding)."""
    bw = max_def.bit_length()
    chunk, metas = b"", []
    for rows, nlev, rep, dfb, plain, enc in pages:
        d = O.hybrid_decode(dfb, bw, nlev) if dfb else np.full(nlev, max_def, np.uint32)
        stream = encode(d[d >= leaf_def], plain, enc)
        body = rows.to_bytes(4, "little") + len(rep).to_bytes(4, "little") + len(dfb).to_bytes(4, "little")
        chunk += body + rep + dfb + stream
        metas.append((len(body) + len(rep) + len(dfb) + len(stream), nlev))
    return chunk, metas


def utf8_stream(slot_def, plain, max_def, opts=None):
    """PLAIN BYTE_ARRAY values ([u32 len][bytes]) of the non-null slots -> a
    compress_binary stream over every leaf slot (null slots empty)."""
    strs, p = [], 0
    for dv in slot_def:
        if dv == max_def:
            n = int.from_bytes(plain[p:p + 4], "little")
            strs.append(plain[p + 4:p + 4 + n])
            p += 4 + n
        else:
            strs.append(b"")
    vals, offs = O.strings_to_arrow(strs)
    return O.write_binary_page(vals, offs, None, False, opts or O.WriteOptions.make())


def bool_stream(slot_def, plain, max_def, opts=None, encoding=0):
    """PLAIN (bit-packed) or RLE ([u32 len][hybrid, bit width 1]) booleans of
    the non-null slots -> a compress_boolean stream over every leaf slot (null
    slots false)."""
    nn = slot_def == max_def
    if encoding == 3:
        bits = O.hybrid_decode(plain[4:4 + int.from_bytes(plain[:4], "little")], 1, int(nn.sum())).astype(bool)
    else:
        bits = np.unpackbits(np.frombuffer(plain, np.uint8), bitorder="little")[:int(nn.sum())].astype(bool)
    v = np.zeros(len(slot_def), bool)
    v[nn] = bits
    return O.write_bool_page(v, None, False, opts or O.WriteOptions.make(), offset=0, n=len(v))


@pytest.mark.parametrize("leaf", ["utf8", "bool"])
@pytest.mark.parametrize("list_nullable", [False, True], ids=["list_req", "list_null"])
@pytest.mark.parametrize("item_nullable", [False, True], ids=["item_req", "item_null"])
def test_list_of_utf8_bool_match_pyarrow(tmp_path, leaf, list_nullable, item_nullable):
    rng = np.random.default_rng(31 + 2 * list_nullable + item_nullable)
    vals = []
    for _ in range(6000):
        r = rng.random()
        if list_nullable and r < 0.1:
            vals.append(None)
        elif r < 0.2:
            vals.append([])
        else:
            k = int(rng.integers(1, 6))
            if leaf == "utf8":
                vals.append([None if item_nullable and rng.random() < 0.15 else str(x) * int(rng.integers(0, 3))
                             for x in rng.integers(0, 10**6, k)])
            else:
                vals.append([None if item_nullable and rng.random() < 0.15 else bool(x) for x in rng.integers(0, 2, k)])
    t_item = pa.utf8() if leaf == "utf8" else pa.bool_()
    field = pa.field("c", pa.list_(pa.field("item", t_item, nullable=item_nullable)), nullable=list_nullable)
    t = pa.table({"c": pa.array(vals, type=field.type)}, schema=pa.schema([field]))
    path = str(tmp_path / "lu.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False,
                   data_page_size=4096, write_statistics=False)
    leaf_def = int(list_nullable) + 1
    max_def = leaf_def + int(item_nullable)
    if leaf == "utf8":
        encode = lambda sd, pl, e: utf8_stream(sd, pl, max_def)  # noqa: E731
    else:
        encode = lambda sd, pl, e: bool_stream(sd, pl, max_def, encoding=e)  # noqa: E731
    chunk, metas = leaf_pages(data_pages_v2(path, True), max_def, leaf_def, encode)
    (offs,), (lv,), values, fv = O.read_nested_column(chunk, metas, np.uint8, (list_nullable,), item_nullable,
                                                      leaf="binary" if leaf == "utf8" else "bool")
    arr = t.column("c").combine_chunks()
    assert (offs == arr.offsets.to_numpy()).all()
    if list_nullable:
        assert (lv == arr.is_valid().to_numpy(zero_copy_only=False)).all()
    items = arr.values
    present = items.is_valid().to_numpy(zero_copy_only=False)
    if item_nullable:
        assert (fv == present).all()
    if leaf == "utf8":
        vo, vb = values
        got = [vb[vo[i]:vo[i + 1]] for i in range(len(vo) - 1)]
        exp = items.to_pylist()
        assert len(got) == len(exp)
        assert all(g == e.encode() for g, e, ok in zip(got, exp, present) if ok)
    else:
        exp = np.array([bool(x) for x in items.to_pylist()], bool) if len(items) else np.zeros(0, bool)
        assert len(values) == len(exp)
        assert (values[present] == exp[present]).all()


# ---- Struct / Map nesting (read/deserialize.rs:140-233) ----------------------
def pages_v2_all(path, col):
    """(rows, levels, rep bytes, def bytes) of every data page of leaf column
    `col` over all row groups."""
    f = pq.ParquetFile(path)
    raw = open(path, "rb").read()
    out = []
    for g in range(f.metadata.num_row_groups):
        cm = f.metadata.row_group(g).column(col)
        p, end = cm.data_page_offset, cm.data_page_offset + cm.total_compressed_size
        while p < end:
            c = Compact(raw, p)
            h = c.struct()
            body = raw[c.p:c.p + h[3]]
            p = c.p + h[3]
            if h[1] != 3:
                continue
            v2 = h[8]
            dl, rl = v2[5], v2[6]
            out.append((v2[3], v2[1], body[:rl], body[rl:rl + dl]))
    return out


STRUCT_SHAPES = ["struct", "map", "list_struct", "list_map", "struct_list", "null_struct", "struct_struct",
                 "list_null_struct_list", "map_of_list", "req_struct_req"]


def _shape(name, n, seed):
    from tests import nestgen

    f = nestgen.shapes()[name]
    f.name = "c"
    a = nestgen.gen(f, n, np.random.default_rng(seed))
    return f, a


@pytest.mark.parametrize("shape", STRUCT_SHAPES)
def test_struct_map_levels_match_pyarrow(tmp_path, shape):
    """The oracle's level writer (oracle.nest.levels: arrow2 to_nested +
    RepLevelsIter / DefLevelsIter) gives pyarrow's parquet levels page for
    page, and the oracle's reader (orc_read_nest_page + create_struct /
    create_map / create_list) turns pyarrow's own level streams back into
    pyarrow's arrays: offsets, validity at every nest, leaf values."""
    from oracle import nest as NE
    from tests import nestgen

    P, n = 700, 3000
    f, a = _shape(shape, n, 100 + STRUCT_SHAPES.index(shape))
    arr = nestgen.to_pa(f, a)
    t = pa.table({"c": arr}, schema=pa.schema([nestgen.pa_field(f)]))
    path = str(tmp_path / "s.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False, row_group_size=P,
                   data_page_size=1 << 30, write_statistics=False)
    paths = NE.leaf_paths(f)
    assert pq.ParquetFile(path).metadata.num_columns == len(paths)
    columns = []
    for c, lp in enumerate(paths):
        max_rep, max_def = NE._max_levels(lp)
        pages = pages_v2_all(path, c)
        assert len(pages) == (n + P - 1) // P
        leaf_a = NE._arrays_on_path(a, lp)[-1]
        chunk, metas = b"", []
        for g, (rows, nlev, rep, dfb) in enumerate(pages):
            r0, r1 = g * P, min(n, (g + 1) * P)
            assert rows == r1 - r0
            ours_rep, ours_def, j0, j1 = NE.levels(a, lp, r0, r1)
            prep = O.hybrid_decode(rep, max_rep.bit_length(), nlev) if max_rep else np.zeros(nlev, np.uint32)
            pdef = O.hybrid_decode(dfb, max_def.bit_length(), nlev) if max_def else np.zeros(nlev, np.uint32)
            assert len(ours_rep) == nlev, (c, g)
            assert (ours_rep == prep).all() and (ours_def == pdef).all(), (c, g)
            # a strawboat page from pyarrow's level bytes + our values section
            body = rows.to_bytes(4, "little") + len(rep).to_bytes(4, "little") + len(dfb).to_bytes(4, "little")
            page = body + rep + dfb + NE.leaf_stream(lp[-1], leaf_a, j0, j1, O.WriteOptions.make())
            chunk += page
            metas.append((len(page), nlev))
        columns.append((chunk, metas))
    got = NE.read_field(f, columns)
    NE.equal(f, got, a, values_under_nulls=True)
    # and the oracle writer's own pages read back the same
    NE.equal(f, NE.read_field(f, NE.write_field(f, a, P)), a, values_under_nulls=True)
