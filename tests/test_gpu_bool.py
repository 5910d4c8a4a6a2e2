"""GPU parity for Boolean columns (read_boolean, read/array/boolean.rs:191-219;
decompress_boolean, compression/boolean/mod.rs:63-102): the HIP page kernel
vs the oracle, bit-exact values bitmap (bits under null slots included) and
validity, through the C ABI.  Pages from the oracle's restatement of
compress_boolean (Basic None/LZ4/Snappy, RLE, OneValue)."""
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


def bool_values(kind, n, rng):
    if kind == "rand":
        return rng.random(n) > 0.5
    if kind == "runs":
        return np.repeat(rng.random(n // 50 + 1) > 0.5, 50)[:n]
    if kind == "long_runs":
        return np.repeat(rng.random(n // 3000 + 1) > 0.5, 3000)[:n]
    if kind == "true":
        return np.ones(n, bool)
    return np.zeros(n, bool)


def oracle_chunk(values, validity, nullable, page_rows, opts):
    pages, metas, row = [], [], 0
    n = len(values)
    while row < n or (n == 0 and not metas):
        m = min(page_rows, n - row)
        pages.append(O.write_bool_page(values, validity[row:row + m] if nullable else None, nullable, opts,
                                       offset=row, n=m))
        metas.append((len(pages[-1]), m))
        row += m
        if n == 0:
            break
    return b"".join(pages), metas


def gpu_bool(ctx, chunk, metas, nullable):
    import pa_amd

    dec = pa_amd.ColumnDecoder(chunk, [pa_amd.PageMeta(l, n) for l, n in metas], np.bool_, nullable, ctx)
    vals, bm = dec.decode()
    n = dec.num_rows
    v = np.unpackbits(vals.cpu().numpy(), bitorder="little")[:n].astype(bool)
    m = np.unpackbits(bm.cpu().numpy(), bitorder="little")[:n].astype(bool) if nullable else None
    dec.close()
    return v, m


OPTS = {
    "plain": dict(),
    "adaptive": dict(ratio=1.2),
    "lz4": dict(default_codec=O.LZ4),
    "snappy": dict(default_codec=O.SNAPPY),
    "zstd": dict(default_codec=O.ZSTD),
    "rle": dict(forced=O.RLE),
}


@pytest.mark.parametrize("opt", list(OPTS))
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
@pytest.mark.parametrize("page_rows", [8192, 1000, 1001, 77])
def test_bool_columns(ctx, opt, nullable, page_rows):
    rng = np.random.default_rng(7)
    for kind in ["rand", "runs", "long_runs", "true", "false"]:
        n = 20000
        v = bool_values(kind, n, rng)
        valid = rng.random(n) > 0.15
        chunk, metas = oracle_chunk(v, valid, nullable, page_rows, O.WriteOptions.make(seed=3, **OPTS[opt]))
        ov, om = O.read_bool_column(chunk, metas, nullable)
        gv, gm = gpu_bool(ctx, chunk, metas, nullable)
        assert (gv == ov).all(), f"values differ ({kind})"
        if nullable:
            assert (gm == om).all(), f"validity differs ({kind})"


@pytest.mark.parametrize("n", [1, 31, 33, 8191, 70000])
def test_bool_ragged_and_large_pages(ctx, n):
    rng = np.random.default_rng(n)
    v = rng.random(n) > 0.3
    valid = rng.random(n) > 0.1
    for opts in [O.WriteOptions.make(), O.WriteOptions.make(forced=O.RLE), O.WriteOptions.make(default_codec=O.LZ4)]:
        chunk, metas = oracle_chunk(v, valid, True, n, opts)
        ov, om = O.read_bool_column(chunk, metas, True)
        gv, gm = gpu_bool(ctx, chunk, metas, True)
        assert (gv == ov).all() and (gm == om).all()


BIG_OPTS = {
    "none": dict(),
    "lz4": dict(default_codec=O.LZ4),
    "zstd": dict(default_codec=O.ZSTD),
    "snappy": dict(default_codec=O.SNAPPY),
    "rle": dict(forced=O.RLE),
    "onevalue": dict(ratio=1.2),
}


@pytest.mark.parametrize("rows", [1 << 20, 3_000_000])
@pytest.mark.parametrize("opt", list(BIG_OPTS))
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_bool_single_page_columns(ctx, rows, opt, nullable):
    """max_page_size = None writes one page per chunk (write/common.rs:54-58):
    a Boolean page of 1M / 3M rows exceeds one workgroup's LDS and decodes
    from HBM, its RLE / general-codec bitmap expanded into the page's region
    (boolean/mod.rs:63-102).  Bit-exact against read_bool_column, both
    nullabilities, every codec the writer can pick."""
    rng = np.random.default_rng(rows + len(opt))
    if opt == "onevalue":
        v = np.ones(rows, bool)
    elif opt == "rle":
        v = np.repeat(rng.random(rows // 37 + 1) > 0.5, rng.integers(1, 75, rows // 37 + 1))[:rows]
        v = np.resize(v, rows)
    else:
        v = np.repeat(rng.random(rows // 8 + 1) > 0.3, 8)[:rows] ^ (rng.random(rows) < 0.02)
    valid = rng.random(rows) > 0.1
    chunk, metas = oracle_chunk(v, valid, nullable, rows, O.WriteOptions.make(seed=5, **BIG_OPTS[opt]))
    assert len(metas) == 1
    ov, om = O.read_bool_column(chunk, metas, nullable)
    gv, gm = gpu_bool(ctx, chunk, metas, nullable)
    bad = np.flatnonzero(gv != ov)
    assert len(bad) == 0, f"{len(bad)} values differ, first at {bad[:5]}"
    if nullable:
        assert (gm == om).all(), "validity differs"


def test_bool_big_pages_beside_small_pages(ctx):
    """Big and small pages in one column, at row offsets that are not
    multiples of 32 (shared bitmap words on both sides of a big page)."""
    rng = np.random.default_rng(4)
    parts, metas, chunks, row = [], [], [], 0
    for rows, opt in [(1001, "rle"), (700_003, "lz4"), (77, "none"), (900_001, "rle"), (5, "zstd"),
                      (650_000, "none"), (800_000, "snappy")]:
        v = np.repeat(rng.random(rows // 5 + 1) > 0.5, 5)[:rows]
        valid = rng.random(rows) > 0.2
        c, m = oracle_chunk(v, valid, True, rows, O.WriteOptions.make(**BIG_OPTS[opt]))
        chunks.append(c)
        metas += m
    chunk = b"".join(chunks)
    ov, om = O.read_bool_column(chunk, metas, True)
    gv, gm = gpu_bool(ctx, chunk, metas, True)
    assert (gv == ov).all() and (gm == om).all()


def test_bool_big_malformed_pages(ctx):
    """The big-page path reports the small path's statuses."""
    import pa_amd

    n = 1_500_000
    good = O.write_bool_page(np.ones(n, bool), None, False, O.WriteOptions.make(forced=O.RLE))
    nb = (n + 7) // 8
    cases = {
        "rle short": good[:9] + (n - 1).to_bytes(4, "little") + b"\x01",
        "rle overshoot": good[:9] + (n + 1).to_bytes(4, "little") + b"\x01",
        "none size": bytes([0]) + (nb - 1).to_bytes(4, "little") + n.to_bytes(4, "little") + b"\xff" * (nb - 1),
        "lz4 garbage": bytes([1]) + (nb).to_bytes(4, "little") + n.to_bytes(4, "little") + b"\xf0" * nb,
    }
    for name, page in cases.items():
        with pytest.raises(pa_amd.StrawboatError):
            gpu_bool(ctx, page, [(len(page), n)], False)
        with pytest.raises(O.OracleError):
            O.read_bool_column(page, [(len(page), n)], False)


def test_bool_product_encoder_roundtrip(ctx):
    import pa_amd

    rng = np.random.default_rng(11)
    n = 100_000
    v = np.repeat(rng.random(n // 40 + 1) > 0.5, 40)[:n]
    valid = rng.random(n) > 0.05
    chunk, metas = pa_amd.encode_column(v, valid, True, pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=8192))
    gv, gm = gpu_bool(ctx, chunk, [(m.length, m.num_values) for m in metas], True)
    assert (gm == valid).all()
    assert (gv[valid] == v[valid]).all()


def test_bool_malformed_pages(ctx):
    import pa_amd

    n = 100
    good = O.write_bool_page(np.ones(n, bool), None, False, O.WriteOptions.make(forced=O.RLE))
    cases = {
        "bad codec": bytes([99]) + good[1:],
        "rle short": good[:9 + 5 - 1],
        "rle overshoot": good[:9] + (200).to_bytes(4, "little") + b"\x01",
        "none size": bytes([0]) + (3).to_bytes(4, "little") + (n).to_bytes(4, "little") + b"\xff\xff\xff",
    }
    for name, page in cases.items():
        with pytest.raises(pa_amd.StrawboatError):
            gpu_bool(ctx, page, [(len(page), n)], False)
        with pytest.raises(O.OracleError):
            O.read_bool_column(page, [(len(page), n)], False)
