"""Pages of 1M rows in one page (the write/common.rs:54-58 default when the
caller sets no page size): the fixed-width HBM-source kernel
(k_decode_global), k_inflate on a 8 MiB LZ4 stream, and a header-only Utf8
None page copied from HBM -- each bit-exact against the oracle.  A Float64
Zstd leaf page whose expansion exceeds the deferred pass's LDS decodes
through k_zinflate (frame read from HBM, output written to the column)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

N = 1 << 20


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def one_page(pa_amd, v, valid, nullable, **kw):
    chunk, metas = pa_amd.encode_column(v, valid, nullable, pa_amd.WriteOptions(max_page_size=0, **kw))
    assert len(metas) == 1
    return chunk, metas


@pytest.mark.parametrize("ratio", [None, 1.2])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_int32_1m_page(ctx, ratio, nullable):
    import pa_amd

    rng = np.random.default_rng(1)
    v = rng.integers(0, 1 << 20, N).astype(np.int32)
    valid = rng.random(N) > 0.1 if nullable else None
    chunk, metas = one_page(pa_amd, v, valid, nullable, default_compress_ratio=ratio)
    got, gm = pa_amd.ColumnDecoder(chunk, metas, np.int32, nullable, ctx).decode()
    ev, em = O.read_column(chunk, [(m.length, m.num_values) for m in metas], np.int32, nullable)
    assert got.cpu().numpy().tobytes() == ev.tobytes()
    if nullable:
        assert (pa_amd.read.unpack_bitmap(gm, N).cpu().numpy() == em).all()


def test_float64_lz4_1m_page(ctx):
    import pa_amd

    rng = np.random.default_rng(2)
    v = np.round(rng.standard_normal(N) * 1e4, 2)
    valid = rng.random(N) > 0.1
    chunk, metas = one_page(pa_amd, v, valid, True, default_compression=1)
    got, gm = pa_amd.ColumnDecoder(chunk, metas, np.float64, True, ctx).decode()
    ev, em = O.read_column(chunk, [(m.length, m.num_values) for m in metas], np.float64, True)
    assert got.cpu().numpy().tobytes() == ev.tobytes()
    assert (pa_amd.read.unpack_bitmap(gm, N).cpu().numpy() == em).all()


@pytest.mark.parametrize("rows", [N, 40_000, 3 << 20])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
@pytest.mark.parametrize("dt", [np.float64, np.int32], ids=["f64", "i32"])
def test_zstd_big_page(ctx, rows, nullable, dt):
    """A Zstd leaf page whose expansion exceeds the deferred pass's LDS:
    k_zinflate, one wave reading the frame from HBM and writing the column."""
    import pa_amd

    rng = np.random.default_rng(3)
    v = np.round(rng.standard_normal(rows) * 1e4, 2) if dt == np.float64 else rng.integers(0, 1 << 20, rows).astype(dt)
    valid = rng.random(rows) > 0.1 if nullable else None
    chunk, metas = one_page(pa_amd, v, valid, nullable, default_compression=2)
    got, gm = pa_amd.ColumnDecoder(chunk, metas, dt, nullable, ctx).decode()
    ev, em = O.read_column(chunk, [(m.length, m.num_values) for m in metas], dt, nullable)
    assert got.cpu().numpy().tobytes() == ev.tobytes()
    if nullable:
        assert (pa_amd.read.unpack_bitmap(gm, rows).cpu().numpy() == em).all()


def test_zstd_big_pages_many(ctx):
    """Several big Zstd pages in one column, each its own k_zinflate job."""
    import pa_amd

    rng = np.random.default_rng(5)
    v = rng.integers(0, 1000, 5 * 65536 + 17).astype(np.int64)
    chunk, metas = pa_amd.encode_column(v, None, False, pa_amd.WriteOptions(default_compression=2, max_page_size=65536))
    assert len(metas) == 6
    got, _ = pa_amd.ColumnDecoder(chunk, metas, np.int64, False, ctx).decode()
    assert (got.cpu().numpy() == v).all()


@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_utf8_none_1m_page(ctx, nullable):
    import pa_amd

    rng = np.random.default_rng(4)
    strs = [str(x).encode() for x in rng.integers(0, 10**9, N)]
    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    valid = rng.random(N) > 0.1 if nullable else None
    chunk, metas = pa_amd.encode_binary_column(vals, offs, valid, nullable, pa_amd.WriteOptions(max_page_size=0))
    assert len(metas) == 1
    go, gv, gm = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, nullable, ctx).decode()
    eo, ev, em = O.read_binary_column(chunk, [(m.length, m.num_values) for m in metas], nullable)
    assert (go.cpu().numpy() == eo).all()
    assert gv.cpu().numpy()[:len(ev)].tobytes() == ev
    if nullable:
        assert (pa_amd.read.unpack_bitmap(gm, N).cpu().numpy() == em).all()


@pytest.mark.parametrize("phys", ["UTF8", "LARGE_UTF8"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_utf8_zstd_big_page(ctx, phys, nullable):
    """A Basic Zstd Utf8 page too large for the staged passes: both streams
    through k_zinflate (offsets via scratch, values at the page's base)."""
    import pa_amd

    rng = np.random.default_rng(6)
    n = 300_000
    strs = [str(x).encode() * int(rng.integers(0, 3)) for x in rng.integers(0, 10**9, n)]
    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    valid = rng.random(n) > 0.1 if nullable else None
    pt = getattr(pa_amd, phys)
    chunk, metas = pa_amd.encode_binary_column(vals, offs, valid, nullable,
                                               pa_amd.WriteOptions(default_compression=2, max_page_size=100_000),
                                               physical_type=pt)
    assert len(metas) == 3
    o, v, m = pa_amd.BinaryColumnDecoder(chunk, metas, pt, nullable, ctx).decode()
    eo, ev, em = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], nullable,
                                      offset_width=8 if phys == "LARGE_UTF8" else 4)
    assert (o.cpu().numpy() == eo).all()
    assert v.cpu().numpy()[:len(ev)].tobytes() == ev
    if nullable:
        assert (pa_amd.read.unpack_bitmap(m, n).cpu().numpy() == em).all()
