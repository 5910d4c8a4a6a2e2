"""Device page encode (sb_encode_column_device) against the host writer and the
oracle: for the options whose codec choice needs no trial compression
(ratio None, default codec None, forced codec none or Bitpacking --
choose_compressor, compression/integer/mod.rs:231-240; bp.rs:92-100) the
device chunk must be byte-identical to sb_encode_column's, its page metas
equal, and it must decode (oracle and GPU) to the input values."""
import zlib

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


BOOL_BIG_OPTS = {
    "none": dict(),
    "lz4": dict(default_compression=1),
    "snappy": dict(default_compression=3),
    "rle": dict(forced_codec=10),
    "adaptive": dict(default_compress_ratio=1.2),
}


@pytest.mark.parametrize("P", [20000, 70001, 1 << 20])
@pytest.mark.parametrize("opt", list(BOOL_BIG_OPTS))
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_big_bool_pages(ctx, P, opt, nullable):
    """Boolean pages over 16384 rows (compress_boolean, boolean/mod.rs:23-61):
    the page's bits, run starts and rebuilt bitmap live in its HBM work area.
    Byte-identical to the host writer, and decoded back (oracle and GPU)."""
    import pa_amd

    rng = np.random.default_rng(P + len(opt))
    n = 2 * P + 13  # three pages; the later ones start off a byte boundary when P % 8 != 0
    if opt == "adaptive":  # long runs (RLE), then a constant stretch (OneValue page)
        v = np.concatenate([np.repeat(rng.random(n // 200 + 1) > 0.5, 200)[: n // 2], np.ones(n - n // 2, bool)])
    else:
        v = np.repeat(rng.random(n // 3 + 1) > 0.5, 3)[:n] ^ (rng.random(n) < 0.05)
    valid = rng.random(n) > 0.1
    opts = pa_amd.WriteOptions(max_page_size=P, **BOOL_BIG_OPTS[opt])
    host, hm = pa_amd.encode_column(v, valid, nullable, opts)
    dev, dm = pa_amd.encode_column_device(torch.from_numpy(v.copy()).cuda(), torch.from_numpy(valid).cuda(), nullable,
                                          opts, ctx=ctx)
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
    assert dev.cpu().numpy().tobytes() == host, "device chunk differs from the host writer's"
    metas = [(m.length, m.num_values) for m in hm]
    ov, om = O.read_bool_column(host, metas, nullable)
    keep = valid if nullable else np.ones(n, bool)
    assert (ov[keep] == v[keep]).all()
    dec = pa_amd.ColumnDecoder(dev, dm, np.bool_, nullable, ctx=ctx)
    gv, _ = dec.decode()
    gv = np.unpackbits(gv.cpu().numpy(), bitorder="little")[:n].astype(bool)
    assert (gv == ov).all()


@pytest.mark.parametrize("P", [65542, 131070, 131077])
def test_big_binary_freq_roaring_tmp(ctx, P):
    """Forced-Freq Utf8 pages whose row counts leave no round-up slack after
    the per-page scratch (P % 8 in {6, 5}): roaring_multi's per-container
    table must sit inside the page's scratch, not the next page's."""
    import pa_amd

    rng = np.random.default_rng(P)
    n = 3 * P + 5
    strs = [b"common" if r < 0.96 else str(x).encode() for r, x in zip(rng.random(n), rng.integers(0, 10**7, n))]
    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    opts = pa_amd.WriteOptions(max_page_size=P, default_compress_ratio=2.0, forced_codec=13)
    valid = rng.random(n) > 0.1
    host, hm = pa_amd.encode_binary_column(vals, offs, valid, True, opts, physical_type=pa_amd.UTF8)
    dev, dm = pa_amd.encode_binary_column_device(torch.from_numpy(np.frombuffer(vals, np.uint8).copy()).cuda(),
                                                 torch.from_numpy(offs).cuda(), torch.from_numpy(valid).cuda(), True,
                                                 opts, pa_amd.UTF8, ctx=ctx)
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
    assert dev.cpu().numpy().tobytes() == host


ZSTD_OPTS = {
    "basic": dict(default_compression=2),
    "adaptive": dict(default_compression=2, default_compress_ratio=1.2),
    "dict": dict(default_compression=2, default_compress_ratio=2.0, forced_codec=11),
    "freq": dict(default_compression=2, default_compress_ratio=2.0, forced_codec=13),
}


def page_codecs(chunk, metas, nullable):
    """the codec byte of every page (after its validity prefix)"""
    out, pos = [], 0
    for m in metas:
        q = pos + (4 + int.from_bytes(chunk[pos:pos + 4], "little") if nullable else 0)
        out.append(chunk[q])
        pos += m.length
    return out


@pytest.mark.parametrize("P", [8192, 70_000, None])
@pytest.mark.parametrize("kind", ["f64", "int32_runs", "int64_freq", "int8"])
@pytest.mark.parametrize("opt", list(ZSTD_OPTS))
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_device_zstd_pages(ctx, P, kind, opt, nullable):
    """Zstd as the default codec (CommonCompression::compress, basic.rs:122-135):
    the device writes Zstd frames transcoded from its LZ4 parse (sb_zstdc.h),
    not libzstd level 3's bytes -- the pages carry the host writer's codec
    choices and row counts, and decode (oracle through libzstd, and the GPU
    reader) to the input values."""
    import pa_amd

    rng = np.random.default_rng(zlib.crc32(repr((P, kind, opt)).encode()))  # (str hashes vary per process)
    n = 150_001
    if kind == "f64":
        v = np.round(rng.standard_normal(n) * 1e3, 1)
    elif kind == "int32_runs":
        v = np.repeat(rng.integers(0, 1 << 30, n // 40 + 1), 40)[:n].astype(np.int32)
    elif kind == "int64_freq":
        v = np.where(rng.random(n) < 0.93, 1 << 40, rng.integers(0, 1 << 50, n)).astype(np.int64)
    else:
        v = rng.integers(-100, 100, n).astype(np.int8)
    valid = rng.random(n) > 0.1
    opts = pa_amd.WriteOptions(max_page_size=P, **ZSTD_OPTS[opt])
    host, hm = pa_amd.encode_column(v, valid, nullable, opts)
    dev, dm = pa_amd.encode_column_device(torch.from_numpy(v.copy()).cuda(), torch.from_numpy(valid).cuda(), nullable,
                                          opts, ctx=ctx)
    got = dev.cpu().numpy().tobytes()
    assert [m.num_values for m in dm] == [m.num_values for m in hm]
    assert sum(m.length for m in dm) == len(got)
    assert page_codecs(got, dm, nullable) == page_codecs(host, hm, nullable)
    metas = [(m.length, m.num_values) for m in dm]
    ov, ovalid = O.read_column(got, metas, v.dtype, nullable)
    keep = valid if nullable else np.ones(n, bool)
    assert ov[keep].tobytes() == v[keep].tobytes()
    if nullable:
        assert (ovalid == valid).all()
    dec = pa_amd.ColumnDecoder(dev, dm, v.dtype, nullable, ctx=ctx)
    gv, _ = dec.decode()
    assert gv.cpu().numpy().view(v.dtype)[:n][keep].tobytes() == v[keep].tobytes()


@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_device_zstd_bool_and_utf8(ctx, nullable):
    """Zstd Boolean pages (the bitmap bytes) and Utf8 pages (offsets and
    values streams) from the device decode to the input."""
    import pa_amd

    rng = np.random.default_rng(21)
    n = 100_003
    valid = rng.random(n) > 0.1
    keep = valid if nullable else np.ones(n, bool)
    for P in (4096, 30_000):
        opts = pa_amd.WriteOptions(max_page_size=P, default_compression=2)
        b = np.repeat(rng.random(n // 5 + 1) > 0.5, 5)[:n]
        dev, dm = pa_amd.encode_column_device(torch.from_numpy(b.copy()).cuda(), torch.from_numpy(valid).cuda(),
                                              nullable, opts, ctx=ctx)
        got = dev.cpu().numpy().tobytes()
        ov, _ = O.read_bool_column(got, [(m.length, m.num_values) for m in dm], nullable)
        assert (ov[keep] == b[keep]).all()
        strs = [b"common" if r < 0.5 else str(x).encode() for r, x in zip(rng.random(n), rng.integers(0, 10**6, n))]
        vals, offs = pa_amd.binary.strings_to_arrow(strs)
        for o in (opts, pa_amd.WriteOptions(max_page_size=P, default_compression=2, default_compress_ratio=1.5)):
            dev, dm = pa_amd.encode_binary_column_device(torch.from_numpy(np.frombuffer(vals, np.uint8).copy()).cuda(),
                                                         torch.from_numpy(offs).cuda(), torch.from_numpy(valid).cuda(),
                                                         nullable, o, pa_amd.UTF8, ctx=ctx)
            got = dev.cpu().numpy().tobytes()
            goffs, gvals, gvalid = O.read_binary_column(got, [(m.length, m.num_values) for m in dm], nullable)
            for i in np.flatnonzero(keep)[::97]:
                assert gvals[goffs[i]:goffs[i + 1]] == strs[i]
            d = pa_amd.BinaryColumnDecoder(dev, dm, pa_amd.UTF8, nullable, ctx=ctx)
            to, tv, _ = d.decode()
            to, tv = to.cpu().numpy(), tv.cpu().numpy().tobytes()
            for i in np.flatnonzero(keep)[::97]:
                assert tv[to[i]:to[i + 1]] == strs[i]


@pytest.mark.parametrize("P", [20000, 65535, 65537, 300_000])
@pytest.mark.parametrize("kind", ["int32_mix", "f64_mix", "int64_freq", "int32_dict"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_big_adaptive_pages(ctx, P, kind, nullable):
    """Pages over 16384 rows with the adaptive cascade (their statistics'
    tables in HBM; over 65535 rows 64-bit table words and roaring bitmaps of
    several containers): byte-identical to the host writer, decoded back."""
    import pa_amd

    rng = np.random.default_rng(P + len(kind))
    n = 2 * P + 777
    if kind == "int32_mix":
        v = np.concatenate([rng.integers(0, 1 << 12, n // 2), np.repeat(rng.integers(0, 1 << 30, n // 64 + 1), 32)])[:n]
        v = v.astype(np.int32)
    elif kind == "f64_mix":
        v = np.concatenate([np.round(rng.standard_normal(n // 2), 1), np.full(n - n // 2, 2.5)])
    elif kind == "int64_freq":
        v = np.where(rng.random(n) < 0.93, 1 << 40, rng.integers(0, 1 << 50, n)).astype(np.int64)
    else:
        v = rng.integers(0, 1000, n).astype(np.int32) * 100_003
    valid = rng.random(n) > 0.1
    for ratio in (1.2, 2.0):
        opts = pa_amd.WriteOptions(default_compress_ratio=ratio, max_page_size=P)
        host, hm = pa_amd.encode_column(v, valid, nullable, opts)
        dev, dm = pa_amd.encode_column_device(torch.from_numpy(v.copy()).cuda(), torch.from_numpy(valid).cuda(),
                                              nullable, opts, ctx=ctx)
        assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
        assert dev.cpu().numpy().tobytes() == host
        # decodes to the input on the valid rows (a null slot's bytes follow the codec: Appendix C)
        ov, ovalid = O.read_column(host, [(m.length, m.num_values) for m in hm], v.dtype, nullable)
        keep = valid if nullable else np.ones(n, bool)
        assert (ov[keep].view(np.uint8).tobytes() == v[keep].view(np.uint8).tobytes())


@pytest.mark.parametrize("codec", [0, 1, 3], ids=["none", "lz4", "snappy"])
@pytest.mark.parametrize("P", [None, 300_000])
def test_big_basic_pages(ctx, codec, P):
    """Basic pages of any size (no statistics): max_page_size None writes the
    whole column as one page (write/common.rs:54-58)."""
    import pa_amd

    rng = np.random.default_rng(codec)
    n = 700_001
    v = np.round(rng.standard_normal(n) * 1e4, 2)
    valid = rng.random(n) > 0.1
    for nullable in (False, True):
        roundtrip(ctx, v, valid, nullable, pa_amd.WriteOptions(default_compression=codec, max_page_size=P))


@pytest.mark.parametrize("opt", ["lz4", "dict", "freq", "adaptive"])
def test_big_binary_pages(ctx, opt):
    """Utf8 pages over 16384 rows: Basic LZ4, Dict, Freq (several roaring
    containers) and adaptive pages, byte-identical to the host writer."""
    import pa_amd

    rng = np.random.default_rng(5)
    P = 300_000 if opt in ("lz4", "freq", "adaptive") else 50_000
    n = 2 * P + 11
    pool = [f"v{i}".encode() for i in range(700)]
    strs = [pool[i] if r < 0.95 else str(x).encode()
            for i, r, x in zip(rng.integers(0, 700, n), rng.random(n), rng.integers(0, 10**7, n))]
    if opt == "freq":
        strs = [s if rng.random() < 0.03 else b"common" for s in strs]
    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    o = {"lz4": dict(default_compression=1), "dict": dict(default_compress_ratio=2.0, forced_codec=11),
         "freq": dict(default_compress_ratio=2.0, forced_codec=13), "adaptive": dict(default_compress_ratio=2.0)}[opt]
    opts = pa_amd.WriteOptions(max_page_size=P, **o)
    valid = rng.random(n) > 0.1
    host, hm = pa_amd.encode_binary_column(vals, offs, valid, True, opts, physical_type=pa_amd.UTF8)
    dev, dm = pa_amd.encode_binary_column_device(torch.from_numpy(np.frombuffer(vals, np.uint8).copy()).cuda(),
                                                 torch.from_numpy(offs).cuda(), torch.from_numpy(valid).cuda(), True,
                                                 opts, pa_amd.UTF8, ctx=ctx)
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
    assert dev.cpu().numpy().tobytes() == host


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


def lz4_shapes(rng, n):
    """byte patterns that exercise every branch of the wave LZ4 search:
    incompressible (long skip steps), short and long matches, self-overlapping
    runs, matches at the 64 KiB distance limit, hash collisions in a batch"""
    return {
        "random": rng.integers(0, 256, n, dtype=np.uint8),
        "zeros": np.zeros(n, np.uint8),
        "period3": np.resize(np.array([1, 2, 3], np.uint8), n),
        "text": np.frombuffer(b"".join(str(x).encode() + b"," for x in rng.integers(0, 10**6, n // 4 + 1)), np.uint8)[:n],
        "runs": np.repeat(rng.integers(0, 256, n // 37 + 1, dtype=np.uint8), 37)[:n],
        "blocks": np.tile(rng.integers(0, 256, 4096, dtype=np.uint8), n // 4096 + 1)[:n],
        "far": np.concatenate([rng.integers(0, 256, 65530, dtype=np.uint8)] * (n // 65530 + 1))[:n],
        "sparse": np.where(rng.random(n) < 0.02, rng.integers(0, 256, n), 0).astype(np.uint8),
        "mixed": np.concatenate([rng.integers(0, 256, n // 2, dtype=np.uint8), np.zeros(n - n // 2, np.uint8)]),
    }


@pytest.mark.parametrize("nbytes", [0, 5, 12, 13, 14, 100, 4096, 16384, 65536, 65544, 65552, 131072])
def test_device_lz4_matches_host(ctx, nbytes):
    """Basic LZ4 pages (ratio None, default codec LZ4): the wave-cooperative
    compressor (sb_lz4c.h lz4_compress_wave) writes the host writer's bytes --
    liblz4's greedy parse -- for every data shape, both table modes (pages
    below / above LZ4_64Klimit = 65547 bytes) and tiny inputs."""
    import pa_amd

    rng = np.random.default_rng(nbytes)
    dt = np.uint8 if nbytes <= 16384 else np.uint64
    for name, b in lz4_shapes(rng, max(nbytes, 8)).items():
        v = np.ascontiguousarray(b[:nbytes]).view(dt)
        opts = pa_amd.WriteOptions(default_compression=1, max_page_size=max(len(v), 1))
        assert roundtrip(ctx, v, np.ones(len(v), bool), False, opts) <= {frozenset({1}), frozenset()}, name


@pytest.mark.parametrize("nbytes", [65535, 65546, 65547, 65548, 200_001])
def test_device_lz4_binary_values_stream(ctx, nbytes):
    """Odd stream sizes around LZ4_64Klimit through a Utf8 page's values
    stream (one row holding the whole blob, and 1000-row pages of it)."""
    import pa_amd

    rng = np.random.default_rng(nbytes)
    for name, b in lz4_shapes(rng, nbytes).items():
        blob = (b % 128).astype(np.uint8).tobytes()  # ASCII: a valid Utf8 column
        for rows in (1, 1000):
            cuts = np.sort(rng.integers(0, nbytes, rows - 1)) if rows > 1 else np.zeros(0, np.int64)
            offs = np.concatenate([[0], cuts, [nbytes]]).astype(np.int64)
            opts = pa_amd.WriteOptions(default_compression=1, max_page_size=rows)
            host, hm = pa_amd.encode_binary_column(blob, offs, None, False, opts, physical_type=pa_amd.UTF8)
            tv = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
            dev, dm = pa_amd.encode_binary_column_device(tv, torch.from_numpy(offs).cuda(), None, False, opts,
                                                         pa_amd.UTF8, ctx=ctx)
            assert dev.cpu().numpy().tobytes() == host, (name, rows)


def test_encode_table_device_concurrent(ctx):
    """encode_table_device: columns in flight on four contexts / streams give
    each column the bytes of its own host encode (and of encode_column_device)."""
    import pa_amd

    rng = np.random.default_rng(12)
    n = 50_000
    f = np.round(rng.standard_normal(n) * 1e4, 2)
    ints = rng.integers(0, 1 << 20, n).astype(np.int32)
    valid = rng.random(n) > 0.1
    strs = [str(x).encode() for x in rng.integers(0, 10**6, n)]
    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    lz4 = pa_amd.WriteOptions(default_compression=1, max_page_size=8192)
    ad = pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=8192)
    cols = [pa_amd.DeviceColumn(torch.from_numpy(f).cuda(), None, False, lz4),
            pa_amd.DeviceColumn(torch.from_numpy(ints).cuda(), torch.from_numpy(valid).cuda(), True, ad),
            pa_amd.DeviceColumn(torch.from_numpy(np.frombuffer(vals, np.uint8).copy()).cuda(), None, False, lz4,
                                torch.from_numpy(offs).cuda(), pa_amd.UTF8),
            pa_amd.DeviceColumn(torch.from_numpy(ints).cuda(), None, False, lz4),
            pa_amd.DeviceColumn(torch.from_numpy(f).cuda(), torch.from_numpy(valid).cuda(), True, ad)]
    hosts = [pa_amd.encode_column(f, None, False, lz4), pa_amd.encode_column(ints, valid, True, ad),
             pa_amd.encode_binary_column(vals, offs, None, False, lz4, physical_type=pa_amd.UTF8),
             pa_amd.encode_column(ints, None, False, lz4), pa_amd.encode_column(f, valid, True, ad)]
    for rep in range(2):
        got = pa_amd.encode_table_device(cols, n_streams=4)
        for (c, m), (h, hm) in zip(got, hosts):
            assert c.cpu().numpy().tobytes() == h
            assert [(x.length, x.num_values) for x in m] == [(x.length, x.num_values) for x in hm]
