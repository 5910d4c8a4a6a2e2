"""The product writer for nested fields (sb_encode_nested_column via
pa_amd.encode_field): encode_chunk's to_nested / to_leaves paging
(write/common.rs:60-115) and write_nested (write/serialize.rs:135-198,
217-232) for any List / LargeList / Map / Struct chain over fixed-width,
Boolean and Binary / Utf8 leaves.  Every leaf chunk must be byte-identical to
the oracle's restatement (oracle.nest.write_field, page p sampled with
sb_page_seed(seed, p)) and read back by the oracle's nested reader to the
written array (Arrow logical equality, as io.rs:473 assert_eq!).  Host only:
the device decode of the same chunks is tests/test_gpu_nested_write.py."""
import numpy as np
import pytest

import pa_amd
from oracle import nest as NE
from oracle import oracle as O
from tests import nestgen

CODECS = {
    "none": dict(),
    "lz4": dict(default_codec=O.LZ4),
    "zstd": dict(default_codec=O.ZSTD),
    "snappy": dict(default_codec=O.SNAPPY),
    "adaptive20": dict(ratio=2.0),  # test_write_read's options (io.rs:427-436)
    "lz4_adaptive": dict(ratio=2.0, default_codec=O.LZ4),
}
SEED = 7


def product_options(codec, page_rows):
    o = CODECS[codec]
    return pa_amd.WriteOptions(default_compression=o.get("default_codec", 0), default_compress_ratio=o.get("ratio"),
                               max_page_size=page_rows or None, seed=SEED)


def write_both(f, a, codec, page_rows):
    got = pa_amd.encode_field(nestgen.pa_amd_field(f), nestgen.host_array(a), product_options(codec, page_rows))
    exp = NE.write_field(f, a, page_rows, O.WriteOptions.make(**CODECS[codec]),
                         page_seed=lambda p: pa_amd.page_seed(SEED, p))
    return got, exp


def check_same(f, got, exp):
    assert len(got) == len(exp) == len(NE.leaf_paths(f))
    for k, ((gc, gm), (ec, em)) in enumerate(zip(got, exp)):
        assert [(m.length, m.num_values) for m in gm] == list(em), f"leaf {k}: page metas differ"
        assert gc == ec, f"leaf {k}: chunk bytes differ"


CASES = ["test_struct", "test_map", "test_list_list", "test_list_struct", "test_list_map", "test_struct_list",
         "list_utf8", "list_bool", "list_list_bool"]


@pytest.mark.parametrize("codec", list(CODECS))
@pytest.mark.parametrize("case", CASES)
def test_io_rs_chunks_byte_identical(case, codec):
    """The reference's nested integration chunks (io.rs:167-278) with
    WRITE_PAGE = 2048-row pages (io.rs:46), every codec option."""
    f, a = nestgen.io_rs_cases(np.random.default_rng(11 + CASES.index(case)))[case]
    got, exp = write_both(f, a, codec, 2048 if a.length > 2048 else 256)
    check_same(f, got, exp)
    back = NE.read_field(f, [(c, [(m.length, m.num_values) for m in ms]) for c, ms in got])
    NE.equal(f, back, nestgen.compact(a), values_under_nulls=False)


SHAPES = ["struct", "map", "list_struct", "list_map", "struct_list", "null_struct", "struct_struct",
          "list_null_struct_list", "map_of_list", "req_struct_req"]


@pytest.mark.parametrize("codec", ["none", "lz4", "adaptive20"])
@pytest.mark.parametrize("shape", SHAPES)
def test_shapes_byte_identical(shape, codec):
    rng = np.random.default_rng(300 + SHAPES.index(shape))
    f = nestgen.shapes()[shape]
    for n, page_rows in ((700, 128), (2500, 0)):
        a = nestgen.gen(f, n, rng, uniq=n // 3 if codec.startswith("adaptive") else None)
        got, exp = write_both(f, a, codec, page_rows)
        check_same(f, got, exp)


def test_list_primitive_matches_list_writer():
    """One list level over a fixed-width leaf: the general writer and
    sb_encode_list_column write the same chunk."""
    rng = np.random.default_rng(3)
    f = nestgen.lst(nestgen.leaf("i64", True), True)
    a = nestgen.gen(f, 5000, rng, uniq=100)
    opts = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=1000, seed=SEED)
    (gc, gm), = pa_amd.encode_field(nestgen.pa_amd_field(f), nestgen.host_array(a), opts)
    lc, lm = pa_amd.encode_list_column(a.offsets, a.children[0].values, a.validity, a.children[0].validity,
                                       True, True, opts)
    assert gc == lc and gm == lm


def test_bool_leaf_slices_at_byte_and_bit_offsets():
    """write_bitmap over a sliced Boolean leaf (boolean/mod.rs:41-52): a page
    whose leaf slots start on a byte boundary hands the parent's bytes to the
    Basic codec (trailing bits of the next page included), else a rebuilt
    bitmap -- both match the oracle and decode to the leaf."""
    rng = np.random.default_rng(4)
    f = nestgen.lst(nestgen.leaf("bool", False), False)
    for lens in (np.full(64, 4), rng.integers(0, 5, 64)):
        offs = np.zeros(len(lens) + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        m = int(offs[-1])
        a = NE.A("list", len(lens), None, offsets=offs, children=[NE.A("leaf", m, None, values=rng.random(m) < 0.5)])
        for codec in ("none", "lz4"):
            got, exp = write_both(f, a, codec, 3)
            check_same(f, got, exp)
            NE.equal(f, NE.read_field(f, [(c, [(x.length, x.num_values) for x in ms]) for c, ms in got]), a)


def test_empty_and_one_row():
    f = nestgen.shapes()["list_null_struct_list"]
    rng = np.random.default_rng(5)
    for n in (0, 1):
        a = nestgen.gen(f, n, rng)
        got, exp = write_both(f, a, "lz4", 16)
        check_same(f, got, exp)


def test_decreasing_offsets_refused():
    f = nestgen.lst(nestgen.leaf("i32", False), False)
    a = NE.A("list", 3, None, offsets=np.array([0, 2, 1, 3], np.int64),
             children=[NE.A("leaf", 3, None, values=np.arange(3, dtype=np.int32))])
    with pytest.raises(pa_amd.StrawboatError) as e:
        pa_amd.encode_field(nestgen.pa_amd_field(f), nestgen.host_array(a))
    assert e.value.status == 6  # SB_E_ARG


def test_native_writer_nested_chunk(tmp_path):
    """NativeWriter::write of a chunk mixing flat and nested fields
    (writer.rs:113-143): the file's columns are the leaves in to_leaves
    order and read back through the oracle."""
    rng = np.random.default_rng(6)
    cases = nestgen.io_rs_cases(rng)
    f, a = cases["test_struct_list"]
    flat = rng.integers(0, 100, a.length).astype(np.int32)
    w = pa_amd.NativeWriter(pa_amd.WriteOptions(default_compression=O.LZ4, default_compress_ratio=2.0,
                                                max_page_size=2048))
    w.start()
    w.write([(flat, None, False), (nestgen.pa_amd_field(f), nestgen.host_array(a))])
    data = w.finish()
    assert len(w.metas) == 1 + len(NE.leaf_paths(f))
    c0 = w.metas[0]
    end = w.metas[1].offset
    vals, _ = O.read_column(data[c0.offset:end], [(p.length, p.num_values) for p in c0.pages], np.int32)
    assert (vals == flat).all()
    cols = []
    for m in w.metas[1:]:
        ln = sum(p.length for p in m.pages)
        cols.append((data[m.offset:m.offset + ln], [(p.length, p.num_values) for p in m.pages]))
    NE.equal(f, NE.read_field(f, cols), nestgen.compact(a), values_under_nulls=False)
