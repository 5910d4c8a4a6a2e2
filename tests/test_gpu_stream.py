"""column_iter_to_arrays' page-at-a-time contract (read/deserialize.rs:
237-253) through the C ABI, decoded in page ranges (pa_amd.iter_page_arrays,
the protocol compat::column_iter_to_arrays follows): arrays come back one
per page in page order; a corrupted page k yields the arrays of pages
0..k-1 -- equal to the oracle's reads of those pages -- and then its error;
every array materialises on the host in the reference's shape
(PageArray.to_host -> HostArray, batch_read.rs:190-209 returns host arrays)
equal to the rows it covers."""
import numpy as np
import pytest

from oracle import nest as NE
from oracle import oracle as O
from tests import nestgen

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def readers(columns):
    import pa_amd

    return [pa_amd.NativeReader(chunk, metas) for chunk, metas in columns]


def corrupt(columns, leaf, k, nested):
    """Page k of one leaf column with an unknown codec byte in its values
    stream header (Compression::from_codec -> OutOfSpec, compression/mod.rs:
    78-80)."""
    import pa_amd

    chunk, metas = columns[leaf]
    start = sum(m.length for m in metas[:k])
    page = bytearray(chunk[start:start + metas[k].length])
    if nested:
        at = 12 + int.from_bytes(page[4:8], "little") + int.from_bytes(page[8:12], "little")
    else:
        at = 0
    page[at] = 99
    out = list(columns)
    out[leaf] = (chunk[:start] + bytes(page) + chunk[start + metas[k].length:], metas)
    assert isinstance(out[leaf][1][0], pa_amd.PageMeta)
    return out


@pytest.mark.parametrize("range_pages", [1, 4, 64])
def test_flat_stream_order_and_bad_page(ctx, range_pages):
    import pa_amd

    rng = np.random.default_rng(1)
    vals = rng.integers(0, 1 << 12, 20 * 500).astype(np.int32)
    chunk, metas = pa_amd.encode_column(vals, None, False,
                                        pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=500))
    fld = pa_amd.Field.leaf(np.int32, False)
    got = [a.to_host().values for a in pa_amd.iter_page_arrays(readers([(chunk, metas)]), fld, ctx, range_pages)]
    assert len(got) == len(metas)
    assert np.array_equal(np.concatenate(got), vals)
    for k in (0, 7, 19):
        bad = corrupt([(chunk, metas)], 0, k, False)
        seen = []
        with pytest.raises(pa_amd.StrawboatError) as e:
            for a in pa_amd.iter_page_arrays(readers(bad), fld, ctx, range_pages):
                seen.append(a.to_host().values)
        assert e.value.status == 1  # OutOfSpec
        assert len(seen) == k
        if k:
            assert np.array_equal(np.concatenate(seen), vals[:500 * k])


@pytest.mark.parametrize("case", ["test_struct_list", "test_list_map", "list_utf8"])
def test_nested_stream_order_and_bad_page(ctx, case):
    """A nested field: every leaf reader advances in step; a bad page in the
    last leaf column stops the stream after the rows of the pages before it."""
    import pa_amd

    f, a = nestgen.io_rs_cases(np.random.default_rng(21))[case]
    pf = nestgen.pa_amd_field(f)
    page_rows = 256
    cols = pa_amd.encode_field(pf, nestgen.host_array(a), pa_amd.WriteOptions(default_compression=O.LZ4,
                                                                              default_compress_ratio=2.0,
                                                                              max_page_size=page_rows))
    n_pages = len(cols[0][1])
    pages = list(pa_amd.iter_page_arrays(readers(cols), pf, ctx, 8))
    assert len(pages) == n_pages
    for p, arr in enumerate(pages):
        r0, r1 = p * page_rows, min(a.length, (p + 1) * page_rows)
        assert arr.length == r1 - r0
        NE.equal(f, arr.to_host(), nestgen._slice(a, r0, r1), values_under_nulls=False)
    k = n_pages // 2
    bad = corrupt(cols, len(cols) - 1, k, True)
    seen = []
    with pytest.raises(pa_amd.StrawboatError):
        for arr in pa_amd.iter_page_arrays(readers(bad), pf, ctx, 8):
            seen.append(arr)
    assert len(seen) == k
    for p, arr in enumerate(seen):
        NE.equal(f, arr.to_host(), nestgen._slice(a, p * page_rows, (p + 1) * page_rows), values_under_nulls=False)


def test_batch_to_host_matches_oracle_bit_exact(ctx):
    """The whole-chunk read materialised on the host equals the oracle's read
    of the same chunks, values under null slots included."""
    import pa_amd

    f, a = nestgen.io_rs_cases(np.random.default_rng(22))["test_map"]
    pf = nestgen.pa_amd_field(f)
    cols = pa_amd.encode_field(pf, nestgen.host_array(a), pa_amd.WriteOptions(default_compress_ratio=2.0,
                                                                              max_page_size=300))
    host = pa_amd.to_host(pf, pa_amd.decode_columns(pf, cols, ctx))
    exp = NE.read_field(f, [(c, [(m.length, m.num_values) for m in ms]) for c, ms in cols])
    NE.equal(f, host, exp, values_under_nulls=True)
