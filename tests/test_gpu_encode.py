"""Device page encode (sb_encode_column_device) against the host writer and the
oracle: for the options whose codec choice needs no trial compression
(ratio None, default codec None, forced codec none or Bitpacking --
choose_compressor, compression/integer/mod.rs:231-240; bp.rs:92-100) the
device chunk must be byte-identical to sb_encode_column's, its page metas
equal, and it must decode (oracle and GPU) to the input values."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def roundtrip(ctx, v, valid, nullable, opts):
    import pa_amd

    host, hm = pa_amd.encode_column(v, valid, nullable, opts)
    tv = torch.from_numpy(v.copy()).cuda()
    tvalid = torch.from_numpy(valid.copy()).cuda() if nullable else None
    dev, dm = pa_amd.encode_column_device(tv, tvalid, nullable, opts, ctx=ctx)
    got = dev.cpu().numpy().tobytes()
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
    assert got == host, "device chunk differs from the host writer's"
    # and it decodes to the input, on the oracle and on the GPU
    ov, ovalid = O.read_column(got, [(m.length, m.num_values) for m in dm], v.dtype, nullable)
    assert ov.tobytes() == v.tobytes()
    dec = pa_amd.ColumnDecoder(dev, dm, v.dtype, nullable, ctx=ctx)
    vals, bm = dec.decode()
    assert vals.cpu().numpy().view(v.dtype)[: len(v)].tobytes() == v.tobytes()
    return {got_codec(got, dm, nullable)}


def got_codec(chunk, metas, nullable):
    codecs, pos = set(), 0
    for m in metas:
        q = pos + (4 + int.from_bytes(chunk[pos:pos + 4], "little") if nullable else 0)
        codecs.add(chunk[q])
        pos += m.length
    return frozenset(codecs)


BP = dict(forced_codec=14)


@pytest.mark.parametrize("dtype", [np.int32, np.uint32])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
@pytest.mark.parametrize("rows", [8192 * 5, 8192 * 3 + 256, 8192 * 2 + 1000, 128, 77])
def test_forced_bitpacking(ctx, dtype, nullable, rows):
    import pa_amd

    rng = np.random.default_rng(rows)
    bits = rng.integers(0, 33, rows // 128 + 1).repeat(128)[:rows]
    v = (rng.integers(0, 2**32, rows, dtype=np.uint64) & ((np.uint64(1) << bits.astype(np.uint64)) - np.uint64(1)))
    v = v.astype(np.uint32).astype(dtype)
    if dtype == np.int32:
        v[rng.random(rows) < 0.0001] = -5  # a negative value makes its page ineligible -> None
    valid = rng.random(rows) > 0.2
    codecs = roundtrip(ctx, v, valid, nullable, pa_amd.WriteOptions(max_page_size=8192, **BP))
    if rows % 128 == 0 and dtype == np.uint32:
        assert codecs == {frozenset({O.BITPACKING})}


@pytest.mark.parametrize("dtype", [np.int8, np.uint16, np.int32, np.int64, np.uint64, np.float32, np.float64])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_none_pages(ctx, dtype, nullable):
    """Compression::None (config 1: Int64, examples/strawboat_write.rs), any width."""
    import pa_amd

    rng = np.random.default_rng(3)
    rows = 8192 * 4 + 333
    v = rng.integers(0, 255, rows * np.dtype(dtype).itemsize, dtype=np.uint8).view(dtype)
    valid = rng.random(rows) > 0.1
    codecs = roundtrip(ctx, v, valid, nullable, pa_amd.WriteOptions(max_page_size=8192))
    assert codecs == {frozenset({0})}
    # forced Bitpacking on a type it does not apply to falls back to None
    roundtrip(ctx, v, valid, nullable, pa_amd.WriteOptions(max_page_size=8192, **BP))


def test_config1_int64_none(ctx):
    """configs[0]: non-nullable Int64, 1M rows, Compression::None."""
    import pa_amd

    v = np.random.default_rng(42).integers(-2**63, 2**63 - 1, 1_000_000, dtype=np.int64)
    assert roundtrip(ctx, v, None, False, pa_amd.WriteOptions(max_page_size=8192)) == {frozenset({0})}


def test_unsupported_options_are_nyi(ctx):
    """Zstd as the default codec (libzstd's compressor is not restated on the
    device) and adaptive pages over 16384 rows report NotYetImplemented."""
    import pa_amd

    tv = torch.arange(40000, dtype=torch.int32, device="cuda")
    for opts in (pa_amd.WriteOptions(default_compression=2), pa_amd.WriteOptions(default_compression=2,
                                                                                  default_compress_ratio=1.2),
                 pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=20000)):
        with pytest.raises(pa_amd.StrawboatError) as e:
            pa_amd.encode_column_device(tv, None, False, opts, ctx=ctx)
        assert e.value.status == 2


def test_page_size_clamped_and_missing_validity(ctx):
    """max_page_size larger than the column (or None) is clamped to the
    column length (write/common.rs:54-58); nullable with no bitmap = all valid."""
    import pa_amd

    rng = np.random.default_rng(8)
    v = rng.integers(0, 1000, 3000).astype(np.int32)
    for mp in (None, 100000):
        roundtrip(ctx, v, np.ones(len(v), bool), False, pa_amd.WriteOptions(max_page_size=mp, **BP))
    host, hm = pa_amd.encode_column(v, None, True, pa_amd.WriteOptions(max_page_size=1024))
    dev, dm = pa_amd.encode_column_device(torch.from_numpy(v).cuda(), None, True,
                                          pa_amd.WriteOptions(max_page_size=1024), ctx=ctx)
    assert dev.cpu().numpy().tobytes() == host
