"""Struct / Map nesting on the GPU (read/deserialize.rs:140-233,
read/array/struct_.rs, map.rs): the reference's integration shapes
test_struct, test_map, test_list_struct, test_list_map and test_struct_list
(tests/it/io.rs:167-278; arrays as io.rs:294-341 builds them) plus null
structs, structs in structs and lists under null structs, written by the
oracle's restatement of the writer (oracle.nest.write_field: to_nested /
to_leaves paging, write_nested levels, the leaf's codec cascade) and decoded
leaf by leaf through the C ABI (sb_plan_nested_column with a struct mask ->
k_nest_walk, then the flat / binary / boolean kernels on the leaf streams),
assembled as create_struct / create_map / create_list do.  Bit-exact against
the oracle's reader (orc_read_nest_page, pinned against pyarrow's levels in
tests/test_pyarrow_nested.py), values under null slots included, and equal to
the written arrays at every valid slot."""
import numpy as np
import pytest

from oracle import nest as NE
from oracle import oracle as O
from tests import nestgen

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SHAPES = ["struct", "map", "list_struct", "list_map", "struct_list", "null_struct", "struct_struct",
          "list_null_struct_list", "map_of_list", "req_struct_req"]
CODECS = {
    "none": dict(),
    "lz4": dict(default_codec=O.LZ4),
    "zstd": dict(default_codec=O.ZSTD),
    "snappy": dict(default_codec=O.SNAPPY),
    "adaptive20": dict(ratio=2.0),  # test_write_read's options (io.rs:427-436)
    "lz4_adaptive": dict(ratio=2.0, default_codec=O.LZ4),
}


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def decode_gpu(ctx, f, columns):
    import pa_amd

    dec = pa_amd.FieldDecoder(nestgen.pa_amd_field(f), [(c, [pa_amd.PageMeta(l, v) for l, v in m])
                                                         for c, m in columns], ctx)
    try:
        return nestgen.device_to_host(f, dec.decode())
    finally:
        dec.close()


@pytest.mark.parametrize("codec", list(CODECS))
@pytest.mark.parametrize("shape", SHAPES)
def test_struct_map_shapes(ctx, shape, codec):
    rng = np.random.default_rng(1000 + SHAPES.index(shape))
    f = nestgen.shapes()[shape]
    for n, page_rows in ((1000, 256), (4000, 2048), (3000, 0)):  # WRITE_PAGE-like, large, one page
        a = nestgen.gen(f, n, rng, uniq=n // 3 if codec.startswith("adaptive") else None)
        columns = NE.write_field(f, a, page_rows, O.WriteOptions.make(**CODECS[codec]))
        exp = NE.read_field(f, columns)
        NE.equal(f, exp, a, values_under_nulls=False)
        got = decode_gpu(ctx, f, columns)
        NE.equal(f, got, exp, values_under_nulls=True)


def test_struct_leaves_disagree_is_out_of_spec(ctx):
    """A struct whose leaf columns page different row counts cannot build
    (StructArray::try_new checks child lengths): refused."""
    import pa_amd

    f = nestgen.shapes()["null_struct"]
    a = nestgen.gen(f, 1000, np.random.default_rng(5))
    cols = NE.write_field(f, a, 500)
    b = nestgen.gen(f, 999, np.random.default_rng(6))
    cols_b = NE.write_field(f, b, 500)
    with pytest.raises(pa_amd.StrawboatError):
        decode_gpu(ctx, f, [cols[0], cols_b[1]])


def test_file_struct_map_fields(ctx, tmp_path):
    """A file of struct / map / list fields (the oracle's writer per leaf,
    footer by pa_amd.assemble_file): StrawboatFile.field rebuilds each
    field from the schema's nest chains and read_field decodes it from the
    file through HBM, equal to the oracle's batch read."""
    import pa_amd

    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(77)
    shapes = nestgen.shapes()
    names = ["struct", "map", "list_map", "struct_list", "struct_struct", "map_of_list"]
    fields, arrays, cols = [], [], []
    for k in names:
        f = shapes[k]
        f.name = k
        a = nestgen.gen(f, 2500, rng)
        fields.append(f)
        arrays.append(a)
        for chunk, metas in NE.write_field(f, a, 1000, O.WriteOptions.make(ratio=2.0, default_codec=O.LZ4)):
            cols.append((chunk, [pa_amd.PageMeta(l, v) for l, v in metas]))
    schema = pa.schema([nestgen.pa_field(f) for f in fields])
    p = tmp_path / "nested.sb"
    p.write_bytes(pa_amd.assemble_file(cols, schema.serialize().to_pybytes()[8:]))
    with pa_amd.StrawboatFile(p) as sf:
        c0 = 0
        for top, (f, a) in enumerate(zip(fields, arrays)):
            k = len(NE.leaf_paths(f))
            exp = NE.read_field(f, [(cols[c][0], [(m.length, m.num_values) for m in cols[c][1]])
                                    for c in range(c0, c0 + k)])
            got = nestgen.device_to_host(f, sf.read_field(top, ctx))
            NE.equal(f, got, exp, values_under_nulls=True)
            NE.equal(f, got, a, values_under_nulls=False)
            c0 += k
