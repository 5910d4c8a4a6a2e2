"""Device adaptive encode (sb_encode_column_device with the reference's full
option set) against the oracle's restatement of the writer, page by page:
page p of a column written with seed S must equal oracle write_page of the
same rows with sampler seed page_seed(S, p) (serialize.rs:52-132 ->
compress_integer / compress_double, compression/integer/mod.rs:35-347,
compression/double/mod.rs:32-347), byte for byte, and the chunk must equal the
host writer's.  Zstd default codecs: the device's frames (sb_zstdc.h) are not
libzstd level 3's bytes, so those columns are checked for the host writer's
pages and codec choices and for decoding (oracle, via libzstd) to the input."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.colgen import gen_values, page_codecs, same_pages_but_zstd

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

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
    "tiny_ratio": dict(ratio=0.0001),
}
INT_TYPES = [np.int32, np.uint32, np.int64, np.uint64, np.int8, np.uint8, np.int16, np.uint16]
KINDS = ["index", "full", "sorted", "one", "runs", "short_runs", "freq"]


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def pa_opts(o: dict, page_rows: int, seed: int = 42, forbidden=(O.PATAS,)):
    import pa_amd

    return pa_amd.WriteOptions(default_compression=o.get("default_codec", 0), default_compress_ratio=o.get("ratio"),
                               max_page_size=page_rows, forbidden_compressions=forbidden,
                               forced_codec=o.get("forced", -1), seed=seed)


def oracle_pages(values, validity, nullable, page_rows, o: dict, seed, forbidden):
    import pa_amd

    n = len(values)
    step = min(page_rows or n, n)
    out = []
    for p, off in enumerate(range(0, n, step)):
        m = min(step, n - off)
        val = None if validity is None else validity[off:off + m]
        opts = O.WriteOptions.make(seed=pa_amd.page_seed(seed, p), forbidden=forbidden,
                                   **{k: v for k, v in o.items()})
        out.append(O.write_page(values[off:off + m], val, nullable, opts))
    return out


def device_encode(ctx, values, validity, nullable, opts):
    import pa_amd

    tv = torch.from_numpy(values.copy()).cuda()
    tvalid = torch.from_numpy(validity.copy()).cuda() if validity is not None else None
    chunk, metas = pa_amd.encode_column_device(tv, tvalid, nullable, opts, ctx=ctx)
    return chunk.cpu().numpy().tobytes(), metas


def check(ctx, values, validity, nullable, page_rows, o: dict, seed=42, forbidden=(O.PATAS,), oracle=True):
    """oracle=False: compare with the host writer only (the f32 Patas repeat
    case, where the writers fall back to Basic and the oracle reproduces the
    reference's undecodable page: DESIGN.md deviation 2)."""
    import pa_amd

    opts = pa_opts(o, page_rows, seed, forbidden)
    got, metas = device_encode(ctx, values, validity, nullable, opts)
    host, hmetas = pa_amd.encode_column(values, validity, nullable, opts)
    if o.get("default_codec") == O.ZSTD:  # decode equivalence (same_pages_but_zstd)
        dm = same_pages_but_zstd(got, metas, host, hmetas, nullable)
        ov, ovalid = O.read_column(got, dm, values.dtype, nullable)
        keep = validity if nullable else np.ones(len(values), bool)
        assert ov[keep].tobytes() == values[keep].tobytes()
        if nullable:
            assert (ovalid == validity).all()
        return set(page_codecs(got, dm, nullable))
    assert got == host
    assert [(m.length, m.num_values) for m in metas] == [(m.length, m.num_values) for m in hmetas]
    if not oracle:
        return set()
    exp = oracle_pages(values, validity if nullable else None, nullable, page_rows, o, seed, forbidden)
    assert [m.length for m in metas] == [len(x) for x in exp]
    pos = 0
    for p, x in enumerate(exp):
        assert got[pos:pos + len(x)] == x, f"page {p} differs (oracle codec {O.page_codec(x, nullable)})"
        pos += len(x)
    return {O.page_codec(x, nullable) for x in exp}


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
        for page_rows in (2048, 8192):
            seen |= check(ctx, values, validity, nullable, page_rows, OPTS[opt])


@pytest.mark.parametrize("dtype", [np.float32, np.float64], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("opt", list(OPTS), ids=str)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_float_columns(ctx, dtype, opt, nullable):
    rng = np.random.default_rng(7)
    for kind in ["index", "full", "one", "runs", "freq"]:
        n = 20000
        values = gen_values(kind, n, dtype, rng)
        validity = (rng.random(n) > 0.3) if nullable else None
        check(ctx, values, validity, nullable, 2048, OPTS[opt])


@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_patas_adaptive(ctx, dtype, nullable):
    """Patas as a candidate and forced (double/patas.rs:37-105), f32 repeats
    falling back to the default codec, and float special values."""
    rng = np.random.default_rng(21)
    n = 20000
    v = (np.cumsum(rng.integers(-1, 2, n)) * 0.5 + 1000).astype(dtype)
    validity = (rng.random(n) > 0.2) if nullable else None
    f32 = dtype == np.float32  # f32 repeats: the writers' Basic fallback (DESIGN.md deviation 2)
    for o in (dict(ratio=1.0), dict(ratio=2.0), dict(ratio=1.0, forced=O.PATAS), dict(ratio=None, forced=O.PATAS),
              dict(ratio=1.0, forced=O.PATAS, default_codec=O.LZ4)):
        check(ctx, v, validity, nullable, 2048, o, forbidden=(), oracle=not f32)
    if f32:  # without exact repeats the f32 pages are Patas and match the oracle
        u = v + np.arange(n, dtype=dtype) * dtype(1e-3)
        check(ctx, u, validity, nullable, 2048, dict(ratio=1.0, forced=O.PATAS), forbidden=())
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.5, -1.5, 1e-300], dtype=dtype)
    w = sp[rng.integers(0, len(sp), n)]
    for o in (dict(ratio=1.0), dict(ratio=1.0, forced=O.DICT), dict(ratio=1.0, forced=O.FREQ),
              dict(ratio=1.0, forced=O.RLE)):
        check(ctx, w, validity, nullable, 4096, o, forbidden=(), oracle=not f32)


@pytest.mark.parametrize("page_rows", [1, 127, 128, 1000, 4095, 16384, 0], ids=lambda r: f"page{r}")
def test_ragged_and_edge_pages(ctx, page_rows):
    """Pages of 1 row, non-multiples of 128, the 16384-row maximum, and a
    single page (max_page_size None -> clamped to the column length)."""
    rng = np.random.default_rng(3)
    n = 700 if page_rows in (1, 0) else 33000
    for dtype in (np.int32, np.uint32, np.int64):
        v = gen_values("index", n, dtype, rng, uniq=50)
        valid = rng.random(n) > 0.5
        for o in (OPTS["adaptive20"], OPTS["force_rle"], OPTS["force_dict"], OPTS["lz4_adaptive"]):
            check(ctx, v, valid, True, page_rows, o)
            check(ctx, v, None, False, page_rows, o)


def test_all_null_and_tiny_pages(ctx):
    rng = np.random.default_rng(5)
    for n in (1, 5, 64, 129, 650, 651):
        v = rng.integers(0, 300, n).astype(np.int32)
        for valid in (np.zeros(n, bool), rng.random(n) > 0.95):
            for o in (OPTS["adaptive20"], OPTS["tiny_ratio"], OPTS["force_freq"], OPTS["force_dict"]):
                check(ctx, v, valid, True, 8192, o)


def test_bitmap_roaring_and_dict_freq_cascade(ctx):
    """Freq with > 4096 exceptions (roaring bitmap container) and the
    Dict -> Freq / Freq -> Dict cascades."""
    rng = np.random.default_rng(11)
    n = 16384
    v = np.where(rng.random(n) < 0.6, 300, rng.integers(0, 20, n)).astype(np.int64)
    check(ctx, v, None, False, 16384, dict(ratio=0.5, forced=O.FREQ))
    w = np.where(rng.random(n) < 0.95, 7, rng.integers(1000, 1010, n)).astype(np.int32)
    check(ctx, w, None, False, 8192, dict(ratio=1.0, forced=O.DICT))
    check(ctx, w, rng.random(n) > 0.1, True, 8192, dict(ratio=1.0, forced=O.FREQ))


@pytest.mark.parametrize("dtype", [np.int32, np.uint32, np.int64, np.int16, np.float64], ids=lambda d: np.dtype(d).name)
def test_sample_ratio_null_slots_read_default(ctx, dtype):
    """Null slots read T::default() in the rebuilt trial sample
    (integer/mod.rs:334-336, double/mod.rs:334-336): the device writer's
    choices follow the zeros, byte-identical to oracle and host writer."""
    from tests.test_roundtrip_cpu import _null_slot_column

    rng = np.random.default_rng(78)
    v, valid = _null_slot_column(20000, dtype, rng)
    for o in (dict(ratio=1.2), dict(ratio=1.0), dict(ratio=2.0, default_codec=O.LZ4)):
        codecs = check(ctx, v, valid, True, 8192, o, forbidden=())
        if dtype == np.int32 and o["ratio"] == 1.2:
            assert O.BITPACKING in codecs
