"""Nested fields written by the product writer and read by the device: the
reference's integration chunks test_struct, test_map, test_list_list,
test_list_struct, test_list_map and test_struct_list (tests/it/io.rs:167-278,
arrays built as io.rs:294-415 builds them) plus List<Utf8>, List<Boolean>
and List<List<Boolean>>, written through pa_amd.encode_field
(sb_encode_nested_column: to_nested / to_leaves paging, write_nested levels,
the leaf's codec cascade -- write/common.rs:60-115, serialize.rs:135-232)
under the four test_write_read codecs with ratio 2.0 (io.rs:417-438), checked
byte for byte against the oracle's writer (oracle.nest.write_field), then
decoded leaf by leaf on the GPU (FieldDecoder -> sb_plan_nested_column /
k_nest_walk + the leaf kernels) bit-exact against the oracle's reader, values
under null slots included, and equal to the written array at every valid
slot (io.rs:473 assert_eq!)."""
import numpy as np
import pytest

from oracle import nest as NE
from oracle import oracle as O
from tests import nestgen

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CASES = ["test_struct", "test_map", "test_list_list", "test_list_struct", "test_list_map", "test_struct_list",
         "list_utf8", "list_bool", "list_list_bool"]
CODECS = {"none": O.NONE, "lz4": O.LZ4, "zstd": O.ZSTD, "snappy": O.SNAPPY}
SEED = 13


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


@pytest.mark.parametrize("codec", list(CODECS))
@pytest.mark.parametrize("case", CASES)
def test_io_rs_nested_write_then_gpu_read(ctx, case, codec):
    import pa_amd

    f, a = nestgen.io_rs_cases(np.random.default_rng(500 + CASES.index(case)))[case]
    page_rows = 2048 if a.length > 2048 else 256  # WRITE_PAGE (io.rs:46); smaller chunks get several pages too
    opts = pa_amd.WriteOptions(default_compression=CODECS[codec], default_compress_ratio=2.0,
                               max_page_size=page_rows, seed=SEED)
    got = pa_amd.encode_field(nestgen.pa_amd_field(f), nestgen.host_array(a), opts)
    exp_cols = NE.write_field(f, a, page_rows, O.WriteOptions.make(default_codec=CODECS[codec], ratio=2.0),
                              page_seed=lambda p: pa_amd.page_seed(SEED, p))
    for (gc, gm), (ec, em) in zip(got, exp_cols):
        assert gc == ec and [(m.length, m.num_values) for m in gm] == list(em)
    dec = pa_amd.FieldDecoder(nestgen.pa_amd_field(f), got, ctx)
    try:
        dev = nestgen.device_to_host(f, dec.decode())
    finally:
        dec.close()
    exp = NE.read_field(f, exp_cols)
    NE.equal(f, dev, exp, values_under_nulls=True)
    NE.equal(f, dev, nestgen.compact(a), values_under_nulls=False)


def test_leaf_counts_disagree_under_inner_list(ctx):
    """struct<a, b: list<struct<x, y>>>: x and y share the inner list nest
    but not with a -- a y column from another array (same top-level rows,
    different inner counts) is refused at every node, not only against the
    first leaf."""
    import pa_amd

    f = nestgen.struct([nestgen.leaf("i32", True, "a"),
                        nestgen.lst(nestgen.struct([nestgen.leaf("i32", True, "x"), nestgen.leaf("i64", True, "y")],
                                                   True, "s"), True, "b")], False)
    a = nestgen.gen(f, 800, np.random.default_rng(1))
    b = nestgen.gen(f, 800, np.random.default_rng(2))
    pf, opts = nestgen.pa_amd_field(f), pa_amd.WriteOptions(max_page_size=256)
    ca = pa_amd.encode_field(pf, nestgen.host_array(a), opts)
    cb = pa_amd.encode_field(pf, nestgen.host_array(b), opts)
    # a round trip first
    dec = pa_amd.FieldDecoder(pf, ca, ctx)
    try:
        NE.equal(f, nestgen.device_to_host(f, dec.decode()), a, values_under_nulls=False)
    finally:
        dec.close()
    with pytest.raises(pa_amd.StrawboatError):
        pa_amd.FieldDecoder(pf, [ca[0], ca[1], cb[2]], ctx)
