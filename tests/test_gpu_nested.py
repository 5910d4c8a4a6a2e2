"""General nesting on the GPU (sb_plan_nested_column / k_nest_walk): a
primitive leaf under 1, 2 or 3 list levels in every nullability, pages built
from pyarrow's parquet Data Page V2 rep / def streams (tests/
test_pyarrow_nested.py) with the leaf values stream under several codecs,
decoded bit-exactly against the oracle's general reader
(orc_read_nested_page, itself pinned against pyarrow)."""
import itertools

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
pa = pytest.importorskip("pyarrow")
pq = pytest.importorskip("pyarrow.parquet")

from tests.test_pyarrow_nested import data_pages_v2  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def nested_values(rng, depth, nulls, leaf_null, n):
    def build(level):
        r = rng.random()
        if nulls[level] and r < 0.1:
            return None
        if r < 0.2:
            return []
        if level == depth - 1:
            return [None if leaf_null and rng.random() < 0.15 else int(x)
                    for x in rng.integers(-10**6, 10**6, int(rng.integers(1, 5)))]
        return [build(level + 1) for _ in range(int(rng.integers(1, 4)))]

    t = pa.int64()
    f = pa.field("item", t, nullable=leaf_null)
    for level in reversed(range(depth)):
        f = pa.field("item" if level else "c", pa.list_(f), nullable=nulls[level])
    return pa.table({"c": pa.array([build(0) for _ in range(n)], type=f.type)}, schema=pa.schema([f]))


def chunk_of(tmp_path, t, depth, nulls, leaf_null, opts, page_size=4096):
    path = str(tmp_path / "n.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False,
                   data_page_size=page_size, write_statistics=False)
    leaf_def = sum(int(x) + 1 for x in nulls)
    max_def = leaf_def + int(leaf_null)
    bw = max_def.bit_length()
    chunk, metas = b"", []
    for rows, nlev, rep, dfb, plain in data_pages_v2(path):
        d = O.hybrid_decode(dfb, bw, nlev) if dfb else np.full(nlev, max_def, np.uint32)
        slot_def = d[d >= leaf_def]
        vals = np.zeros(len(slot_def), np.int64)
        nn = slot_def == max_def
        vals[nn] = np.frombuffer(plain, np.int64, int(nn.sum()))
        stream = O.compress(vals, None, opts)
        body = rows.to_bytes(4, "little") + len(rep).to_bytes(4, "little") + len(dfb).to_bytes(4, "little")
        chunk += body + rep + dfb + stream
        metas.append((len(body) + len(rep) + len(dfb) + len(stream), nlev))
    return chunk, metas


CODECS = {"none": dict(), "lz4": dict(default_codec=O.LZ4), "adaptive": dict(ratio=1.2)}


@pytest.mark.parametrize("depth", [1, 2, 3])
@pytest.mark.parametrize("codec", list(CODECS))
def test_nested_depths(ctx, tmp_path, depth, codec):
    import pa_amd

    for nulls in itertools.product([False, True], repeat=depth):
        for leaf_null in (False, True):
            rng = np.random.default_rng(depth * 100 + sum(nulls) * 10 + leaf_null)
            t = nested_values(rng, depth, nulls, leaf_null, 3000)
            chunk, metas = chunk_of(tmp_path, t, depth, nulls, leaf_null, O.WriteOptions.make(**CODECS[codec]))
            eo, eb, ev, ef = O.read_nested_column(chunk, metas, np.int64, nulls, leaf_null)
            dec = pa_amd.NestedColumnDecoder(chunk, [pa_amd.PageMeta(l, m) for l, m in metas], np.int64, nulls,
                                             leaf_null, ctx)
            go, gb, gv, gf = dec.decode()
            for d in range(depth):
                assert (go[d].cpu().numpy().astype(np.int64) == eo[d]).all(), (nulls, leaf_null, d)
                if nulls[d]:
                    n = len(eo[d]) - 1
                    assert (pa_amd.read.unpack_bitmap(gb[d], n).cpu().numpy() == eb[d]).all(), (nulls, d)
            assert (gv.cpu().numpy()[:len(ev)] == ev).all()
            if leaf_null:
                assert (pa_amd.read.unpack_bitmap(gf, len(ev)).cpu().numpy() == ef).all()
            dec.close()


@pytest.mark.parametrize("leaf", ["utf8", "bool"])
@pytest.mark.parametrize("depth", [1, 2])
@pytest.mark.parametrize("codec", ["none", "lz4", "adaptive"])
def test_nested_utf8_bool_leaves(ctx, tmp_path, leaf, depth, codec):
    """List<Utf8>, List<Boolean> (and one level deeper): the level walk, then
    the leaf's values streams through the binary / boolean kernels at their
    leaf bases, against the oracle's general reader."""
    import pa_amd
    from tests.test_pyarrow_nested import bool_stream, leaf_pages, utf8_stream

    opts = O.WriteOptions.make(**CODECS[codec])
    for nulls in itertools.product([False, True], repeat=depth):
        for leaf_null in (False, True):
            rng = np.random.default_rng(7 + depth * 10 + sum(nulls) + 3 * leaf_null)

            def build(level):
                r = rng.random()
                if nulls[level] and r < 0.1:
                    return None
                if r < 0.2:
                    return []
                k = int(rng.integers(1, 5))
                if level == depth - 1:
                    if leaf == "utf8":
                        return [None if leaf_null and rng.random() < 0.15 else str(x) * int(rng.integers(0, 3))
                                for x in rng.integers(0, 1000, k)]
                    return [None if leaf_null and rng.random() < 0.15 else bool(x) for x in rng.integers(0, 2, k)]
                return [build(level + 1) for _ in range(k)]

            f = pa.field("item", pa.utf8() if leaf == "utf8" else pa.bool_(), nullable=leaf_null)
            for level in reversed(range(depth)):
                f = pa.field("item" if level else "c", pa.list_(f), nullable=nulls[level])
            t = pa.table({"c": pa.array([build(0) for _ in range(3000)], type=f.type)}, schema=pa.schema([f]))
            path = str(tmp_path / "u.parquet")
            pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False,
                           data_page_size=4096, write_statistics=False)
            leaf_def = sum(int(x) + 1 for x in nulls)
            max_def = leaf_def + int(leaf_null)
            if leaf == "utf8":
                enc = lambda sd, pl, e: utf8_stream(sd, pl, max_def, opts)  # noqa: E731
            else:
                enc = lambda sd, pl, e: bool_stream(sd, pl, max_def, opts, encoding=e)  # noqa: E731
            chunk, metas = leaf_pages(data_pages_v2(path, True), max_def, leaf_def, enc)
            eo, eb, ev, ef = O.read_nested_column(chunk, metas, np.uint8, nulls, leaf_null,
                                                  leaf="binary" if leaf == "utf8" else "bool")
            pm = [pa_amd.PageMeta(l, m) for l, m in metas]
            if leaf == "utf8":
                dec = pa_amd.NestedColumnDecoder(chunk, pm, np.uint8, nulls, leaf_null, ctx, physical_type=pa_amd.UTF8)
            else:
                dec = pa_amd.NestedColumnDecoder(chunk, pm, np.bool_, nulls, leaf_null, ctx)
            go, gb, gv, gf = dec.decode()
            for d in range(depth):
                assert (go[d].cpu().numpy().astype(np.int64) == eo[d]).all(), (nulls, leaf_null, d)
                if nulls[d]:
                    assert (pa_amd.read.unpack_bitmap(gb[d], len(eo[d]) - 1).cpu().numpy() == eb[d]).all()
            nleaf = len(eo[-1]) and int(eo[-1][-1])
            if leaf == "utf8":
                lo, vb = gv
                assert (lo.cpu().numpy().astype(np.int64) == ev[0]).all()
                assert vb.cpu().numpy()[:len(ev[1])].tobytes() == ev[1]
            else:
                assert (pa_amd.read.unpack_bitmap(gv, nleaf).cpu().numpy() == ev).all()
            if leaf_null:
                assert (pa_amd.read.unpack_bitmap(gf, nleaf).cpu().numpy() == ef).all()
            dec.close()


def hybrid_runs(stream: bytes, bw: int) -> int:
    """Run headers of a parquet RLE / bit-packed hybrid stream."""
    p, runs = 0, 0
    while p < len(stream):
        h, sh = 0, 0
        while True:
            c = stream[p]
            p += 1
            h |= (c & 0x7F) << sh
            sh += 7
            if not c & 0x80:
                break
        p += (h >> 1) * bw if h & 1 else (bw + 7) // 8
        runs += 1
    return runs


@pytest.mark.parametrize("list_null", [False, True])
@pytest.mark.parametrize("leaf_null", [False, True])
def test_list_decoder_many_hybrid_runs(ctx, tmp_path, list_null, leaf_null):
    """pyarrow's writer mixes RLE and bit-packed runs within a level stream;
    a page whose rep / def streams hold more runs than the List kernels'
    run table (64) is planned on the general level walk (k_nest_walk), as
    parquet2's HybridRleDecoder takes any number of runs (read_basic.rs:
    83-85).  ListColumnDecoder output == the oracle's reader."""
    import pa_amd

    rng = np.random.default_rng(31 + 2 * list_null + leaf_null)
    rows = []
    for seg in range(400):  # constant stretches (RLE runs) between random ones (bit-packed runs)
        if seg % 2:
            rows += [[int(x)] for x in rng.integers(0, 1000, 40)]
        else:
            for _ in range(25):
                r = rng.random()
                rows.append(None if list_null and r < 0.1 else [] if r < 0.25 else
                            [None if leaf_null and rng.random() < 0.2 else int(x) for x in rng.integers(0, 1000, 2)])
    f = pa.field("c", pa.list_(pa.field("item", pa.int64(), nullable=leaf_null)), nullable=list_null)
    t = pa.table({"c": pa.array(rows, type=f.type)}, schema=pa.schema([f]))
    chunk, metas = chunk_of(tmp_path, t, 1, (list_null,), leaf_null, O.WriteOptions.make(), page_size=1 << 20)
    max_def = 2 + int(list_null) + int(leaf_null) - 1
    pos, most = 0, 0
    for length, nlev in metas:
        rep_len = int.from_bytes(chunk[pos + 4:pos + 8], "little")
        def_len = int.from_bytes(chunk[pos + 8:pos + 12], "little")
        rep = chunk[pos + 12:pos + 12 + rep_len]
        dfb = chunk[pos + 12 + rep_len:pos + 12 + rep_len + def_len]
        most = max(most, hybrid_runs(rep, 1), hybrid_runs(dfb, max_def.bit_length()) if def_len else 0)
        pos += length
    assert most > 64, most
    eo, eb, ev, ef = O.read_nested_column(chunk, metas, np.int64, (list_null,), leaf_null)
    dec = pa_amd.ListColumnDecoder(chunk, [pa_amd.PageMeta(l, m) for l, m in metas], np.int64, list_null, leaf_null,
                                   ctx)
    assert dec.num_rows == len(eo[0]) - 1 and dec.num_leaves == len(ev)
    go, gl, gv, gf = dec.decode()
    assert (go.cpu().numpy().astype(np.int64) == eo[0]).all()
    if list_null:
        assert (pa_amd.read.unpack_bitmap(gl, dec.num_rows).cpu().numpy() == eb[0]).all()
    assert (gv.cpu().numpy()[:len(ev)] == ev).all()
    if leaf_null:
        assert (pa_amd.read.unpack_bitmap(gf, len(ev)).cpu().numpy() == ef).all()
    dec.close()
