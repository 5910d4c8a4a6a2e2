"""GPU parity: batched HIP page decode vs the oracle, bit-exact (values bytes
under null slots included, validity bits), through the C ABI.

Pages come from the oracle's restatement of the reference writer
(serialize.rs:52-132 + compress_integer / compress_double with adaptive
selection, forced codecs as util/env.rs would force them)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.colgen import build_column, gen_values, oracle_decode_column

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def gpu_decode(ctx, chunk, metas, dtype, nullable):
    import pa_amd

    pm = [pa_amd.PageMeta(l, n) for l, n in metas]
    dec = pa_amd.ColumnDecoder(chunk, pm, dtype, nullable, ctx)
    vals, bm = dec.decode()
    n = dec.num_rows
    v = vals.cpu().numpy().view(np.uint8)[: n * np.dtype(dtype).itemsize].view(dtype)
    valid = None
    if nullable:
        valid = np.unpackbits(bm.cpu().numpy(), bitorder="little")[:n].astype(bool)
    dec.close()
    return v, valid


def check(ctx, values, validity, nullable, page_rows, opts):
    dtype = values.dtype
    chunk, metas, codecs = build_column(values, validity, nullable, page_rows, opts)
    ov, om = oracle_decode_column(chunk, metas, dtype, nullable)
    gv, gm = gpu_decode(ctx, chunk, metas, dtype, nullable)
    assert gv.view(np.uint8).tobytes() == ov.view(np.uint8).tobytes(), f"values differ (codecs {set(codecs)})"
    if nullable:
        assert (gm == om).all(), "validity differs"
    return codecs


NO_PATAS = (O.PATAS,)
OPTS = {
    "plain": dict(ratio=None),
    "adaptive12": dict(ratio=1.2),
    "adaptive20": dict(ratio=2.0),
    "force_freq": dict(ratio=2.0, forced=O.FREQ),
    "force_dict": dict(ratio=2.0, forced=O.DICT),
    "force_rle": dict(ratio=2.0, forced=O.RLE),
    "force_bp": dict(ratio=2.0, forced=O.BITPACKING),
    "lz4": dict(ratio=None, default_codec=O.LZ4),
    "lz4_adaptive": dict(ratio=1.2, default_codec=O.LZ4),
    "snappy": dict(ratio=None, default_codec=O.SNAPPY),
    "snappy_dict": dict(ratio=2.0, default_codec=O.SNAPPY, forced=O.DICT),
    "zstd": dict(ratio=None, default_codec=O.ZSTD),
    "zstd_adaptive": dict(ratio=1.2, default_codec=O.ZSTD),
}

INT_TYPES = [np.int32, np.uint32, np.int64, np.uint64, np.int8, np.uint8, np.int16, np.uint16]
KINDS = ["index", "full", "sorted", "one", "runs", "short_runs", "freq"]


@pytest.mark.parametrize("dtype", INT_TYPES, ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("opt", list(OPTS), ids=str)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_int_columns(ctx, dtype, opt, nullable):
    rng = np.random.default_rng(42)
    seen = set()
    for kind in KINDS:
        n = 20000
        values = gen_values(kind, n, dtype, rng)
        validity = (rng.random(n) > 0.2) if nullable else None
        opts = O.WriteOptions.make(forbidden=NO_PATAS, **OPTS[opt])
        for page_rows in (2048, 8192):
            seen |= set(check(ctx, values, validity, nullable, page_rows, opts))
    assert seen


@pytest.mark.parametrize("dtype", [np.float32, np.float64], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("opt", ["plain", "adaptive12", "adaptive20", "force_freq", "force_dict", "force_rle",
                                 "lz4", "lz4_adaptive", "snappy", "zstd"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_float_columns(ctx, dtype, opt, nullable):
    rng = np.random.default_rng(7)
    for kind in ["index", "full", "one", "runs", "freq"]:
        n = 20000
        values = gen_values(kind, n, dtype, rng)
        validity = (rng.random(n) > 0.3) if nullable else None
        opts = O.WriteOptions.make(forbidden=NO_PATAS, **OPTS[opt])
        check(ctx, values, validity, nullable, 2048, opts)


@pytest.mark.parametrize("page_rows", [1000, 1, 127, 4095, 0], ids=lambda r: f"page{r}")
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_ragged_pages(ctx, page_rows, nullable):
    """Row offsets that are not multiples of 4 / 32 (unaligned outputs and
    validity words shared by two pages); page_rows=0 = one page."""
    rng = np.random.default_rng(3)
    for dtype in (np.int32, np.int64, np.int8):
        n = 5003 if page_rows != 1 else 300
        values = gen_values("index", n, dtype, rng, uniq=50)
        validity = (rng.random(n) > 0.5) if nullable else None
        for opt in ("plain", "adaptive20", "force_rle"):
            opts = O.WriteOptions.make(**OPTS[opt])
            check(ctx, values, validity, nullable, page_rows, opts)


@pytest.mark.parametrize("b", list(range(0, 33)))
def test_bitpack_every_width(ctx, b):
    """Int32/UInt32 Bitpacking pages at every num_bits 0..32 (bp.rs:67-86)."""
    rng = np.random.default_rng(100 + b)
    n = 8192 * 3
    hi = 1 << b
    v = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32) if b else np.zeros(n, np.uint32)
    if b:
        v[::128] |= np.uint32(1 << (b - 1))  # every block really has width b
    opts = O.WriteOptions.make(ratio=0.0001, forced=O.BITPACKING)
    codecs = check(ctx, v, None, False, 8192, opts)
    assert set(codecs) == {O.BITPACKING}
    check(ctx, v.view(np.int32) & np.int32(0x7FFFFFFF), None, False, 8192, opts)


def test_bitpack_mixed_widths(ctx):
    """Per-block widths that change every block: the speculative header walk
    falls back to one block per round."""
    rng = np.random.default_rng(5)
    n = 8192 * 2
    v = np.zeros(n, np.uint32)
    for k in range(n // 128):
        b = int(rng.integers(0, 33))
        blk = rng.integers(0, 1 << b, 128, dtype=np.uint64).astype(np.uint32) if b else np.zeros(128, np.uint32)
        if b:
            blk[0] |= np.uint32(1 << (b - 1))
        v[k * 128:(k + 1) * 128] = blk
    opts = O.WriteOptions.make(ratio=0.0001, forced=O.BITPACKING)
    assert set(check(ctx, v, None, False, 8192, opts)) == {O.BITPACKING}


def test_delta_bitpacking(ctx):
    """Sorted UInt32 -> DeltaBitpacking (delta_bp.rs:69-92): page-wide prefix."""
    rng = np.random.default_rng(9)
    n = 8192 * 4
    v = np.cumsum(rng.integers(0, 1000, n)).astype(np.uint32)
    opts = O.WriteOptions.make(ratio=1.0, forbidden=(O.DICT, O.FREQ, O.RLE, O.ONE_VALUE))
    codecs = check(ctx, v, None, False, 8192, opts)
    assert O.DELTA_BITPACKING in codecs
    # large deltas wrap u32
    v2 = np.cumsum(rng.integers(0, 2**20, n)).astype(np.uint64).astype(np.uint32)
    v2.sort()
    check(ctx, v2, None, False, 8192, opts)


def test_big_pages_global_path(ctx):
    """Pages larger than the LDS stage go through the HBM-source kernel."""
    rng = np.random.default_rng(11)
    for dtype, kind in [(np.int32, "full"), (np.int64, "index"), (np.uint32, "bits20")]:
        n = 40000
        v = gen_values(kind, n, dtype, rng)
        validity = rng.random(n) > 0.1
        check(ctx, v, validity, True, 0, O.WriteOptions.make(ratio=1.2))
        check(ctx, v, None, False, 0, O.WriteOptions.make(ratio=None))


def test_malformed_pages_report_errors(ctx):
    """Corrupt pages give a status, not a crash (reference: Err or panic)."""
    import pa_amd

    rng = np.random.default_rng(1)
    v = gen_values("bits12", 8192, np.uint32, rng)
    page = bytearray(O.write_page(v, None, False, O.WriteOptions.make(ratio=1.2)))
    assert page[0] == O.BITPACKING
    bad_codec = bytearray(page)
    bad_codec[0] = 99  # unknown codec -> OutOfSpec (compression/mod.rs:78-80)
    truncated = page[: len(page) // 2]
    truncated[1:5] = (len(truncated) - 9).to_bytes(4, "little")
    wide = bytearray(page)
    wide[9] = 40  # num_bits > 32
    for bad in (bad_codec, truncated, wide):
        with pytest.raises(pa_amd.StrawboatError):
            gpu_decode(ctx, bytes(bad), [(len(bad), 8192)], np.uint32, False)


@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_patas(ctx, dtype, nullable):
    """Patas pages (double/patas.rs:107-132): slowly varying values, repeats
    (f64 only: the reference's f32 repeat desync), nulls."""
    rng = np.random.default_rng(21)
    n = 20000
    v = (np.cumsum(rng.standard_normal(n)) * 10).astype(dtype)
    if dtype == np.float64:
        v[::7] = v[::7][0]  # exact repeats -> reference back-references
    else:
        v = v + np.arange(n, dtype=dtype) * dtype(1e-3)  # no exact repeats
    validity = (rng.random(n) > 0.2) if nullable else None
    opts = O.WriteOptions.make(ratio=1.0, forced=O.PATAS)
    codecs = check(ctx, v, validity, nullable, 2048, opts)
    assert set(codecs) == {O.PATAS}
    # Patas also under Freq exceptions of a double column
    f = np.where(rng.random(n) < 0.93, dtype(2.5), v)
    check(ctx, f, validity, nullable, 4096, O.WriteOptions.make(ratio=1.0, forced=O.FREQ))


def test_lz4_compressible_and_long_matches(ctx):
    """LZ4 pages with many short matches, overlapping matches (offset < length)
    and long literal runs."""
    rng = np.random.default_rng(8)
    for v in [np.repeat(rng.integers(0, 1000, 3000), 7)[:20000].astype(np.int64),
              np.tile(np.arange(3, dtype=np.int32), 7000),
              rng.integers(-2**31, 2**31 - 1, 20000).astype(np.int32),
              np.zeros(20000, np.int8)]:
        for dc in (O.LZ4, O.SNAPPY):
            check(ctx, v, None, False, 8192, O.WriteOptions.make(default_codec=dc))
            check(ctx, v, rng.random(len(v)) > 0.5, True, 2048, O.WriteOptions.make(default_codec=dc))
