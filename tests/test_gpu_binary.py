"""GPU parity for Binary / Utf8 columns (compression/binary/mod.rs:95-183,
read/array/binary.rs:223-265): offsets, values bytes and validity bit-exact
against the oracle's restatement of read_binary, including the bytes under
null rows (Dict: the previous row's entry; Freq/OneValue: the top value)."""
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


def strings(kind, n, rng):
    if kind == "rand":
        return [str(x).encode() for x in rng.integers(0, 10**6, n)]
    if kind == "low":
        return [str(x).encode() for x in rng.integers(0, 8, n)]
    if kind == "one":
        return [b"abc"] * n
    if kind == "empty":
        return [b"" if rng.random() < 0.5 else b"x" for _ in range(n)]
    if kind == "long":
        return [bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8)) for _ in range(n)]
    return [b"hello" if rng.random() < 0.95 else str(x).encode() for x in rng.integers(0, 1000, n)]


def check(ctx, s, validity, nullable, page_rows, opts, phys):
    import pa_amd

    ow = 8 if phys in (pa_amd.LARGE_BINARY, pa_amd.LARGE_UTF8) else 4
    vals, offs = pa_amd.binary.strings_to_arrow(s)
    pages, metas = [], []
    for i in range(0, len(s), page_rows):
        m = min(page_rows, len(s) - i)
        pg = O.write_binary_page(vals, offs[i:i + m + 1], None if validity is None else validity[i:i + m], nullable,
                                 opts, offset_width=ow, parent_values_len=len(vals))
        pages.append(pg)
        metas.append((len(pg), m))
    chunk = b"".join(pages)
    eo, ev, evv = O.read_binary_column(chunk, metas, nullable, ow)
    dec = pa_amd.BinaryColumnDecoder(chunk, [pa_amd.PageMeta(l, m) for l, m in metas], phys, nullable, ctx)
    go, gv, gm = dec.decode()
    go = go.cpu().numpy().astype(np.int64)
    gv = gv.cpu().numpy().tobytes()[: dec.values_bytes]
    assert dec.values_bytes == len(ev)
    bad = np.flatnonzero(go != eo)
    assert len(bad) == 0, f"{len(bad)} offsets differ, first at {bad[:4]}: {go[bad[:4]]} vs {eo[bad[:4]]}"
    same = gv == ev
    assert same, "values differ"
    if nullable:
        g = np.unpackbits(gm.cpu().numpy(), bitorder="little")[: len(s)].astype(bool)
        assert (g == evv).all(), "validity differs"
    dec.close()
    return {pg[4 + int.from_bytes(pg[:4], "little")] if nullable else pg[0] for pg in pages}


OPTS = {
    "plain": dict(),
    "lz4": dict(default_codec=O.LZ4),
    "snappy": dict(default_codec=O.SNAPPY),
    "adaptive": dict(ratio=2.0),
    "dict": dict(ratio=2.0, forced=O.DICT),
    "dict_snappy": dict(ratio=2.0, forced=O.DICT, default_codec=O.SNAPPY),
    "freq": dict(ratio=2.0, forced=O.FREQ),
    "zstd": dict(default_codec=O.ZSTD),
    "dict_zstd": dict(ratio=2.0, forced=O.DICT, default_codec=O.ZSTD),
}


@pytest.mark.parametrize("kind", ["rand", "low", "one", "empty", "freq", "long"])
@pytest.mark.parametrize("opt", list(OPTS))
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
@pytest.mark.parametrize("phys", [13, 12], ids=["utf8", "large_binary"])
def test_binary_columns(ctx, kind, opt, nullable, phys):
    rng = np.random.default_rng(17)
    n = 6000
    s = strings(kind, n, rng)
    validity = (rng.random(n) > 0.2) if nullable else None
    page_rows = 256 if kind == "long" else 2048
    if kind == "long" and phys == 13:  # random bytes are not UTF-8 (tests/test_gpu_utf8.py): read as Binary
        phys = 11
    assert check(ctx, s, validity, nullable, page_rows, O.WriteOptions.make(**OPTS[opt]), phys)


def test_binary_page_over_lds_budget(ctx):
    """A Basic None page larger than one workgroup's LDS (≈300 KiB here) is a
    header-only page: offsets and values are copied from HBM (k_bin_light_out)."""
    rng = np.random.default_rng(2)
    s = strings("long", 2048, rng)
    check(ctx, s, None, False, 2048, O.WriteOptions.make(), 11)
    v = rng.random(2048) > 0.3
    check(ctx, s, v, True, 2048, O.WriteOptions.make(), 11)


@pytest.mark.parametrize("entries,width", [(800, 200), (1500, 200)], ids=["160KiB", "300KiB"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_binary_dict_page_over_lds_budget(ctx, entries, width, nullable):
    """A Dict page whose dictionary (160 / 300 KiB) plus expansion exceeds one
    workgroup's LDS is a big page: read from HBM, its entry table and indices
    in the page's HBM region (binary/dict.rs:95-141), bit-exact."""
    rng = np.random.default_rng(2)
    s = [bytes(rng.integers(0, 256, width, dtype=np.uint8)) for _ in range(entries)] * 4
    v = rng.random(len(s)) > 0.2 if nullable else None
    assert check(ctx, s, v, nullable, len(s), O.WriteOptions.make(ratio=2.0, forced=O.DICT), 11) == {11}


@pytest.mark.parametrize("opt", ["dict", "dict_lz4", "dict_zstd", "freq", "one"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_binary_1m_row_single_page(ctx, opt, nullable):
    """One page over 1M rows (write/common.rs:54-58 with no max_page_size):
    Dict (indices bitpacked, LZ4, Zstd -- 4 MiB of indices), Freq (16 roaring
    containers, bitmap ones) and OneValue, each a big page."""
    rng = np.random.default_rng(21)
    n = 1 << 20
    pool = [f"category-{i:04d}".encode() for i in range(300)]
    if opt == "freq":
        s = [b"common-value" if r < 0.91 else str(x).encode() for r, x in zip(rng.random(n), rng.integers(0, 10**6, n))]
    elif opt == "one":
        s = [b"constant"] * n
    else:
        s = [pool[i] for i in rng.integers(0, 300, n)]
    v = rng.random(n) > 0.1 if nullable else None
    o = {"dict": dict(ratio=2.0, forced=O.DICT), "dict_lz4": dict(forced=O.DICT, default_codec=O.LZ4),
         "dict_zstd": dict(forced=O.DICT, default_codec=O.ZSTD), "freq": dict(ratio=2.0, forced=O.FREQ),
         "one": dict(ratio=2.0)}[opt]
    codecs = check(ctx, s, v, nullable, n, O.WriteOptions.make(**o), 13)
    assert codecs == {{"freq": 13, "one": 12}.get(opt, 11)}


@pytest.mark.parametrize("codec", ["lz4", "zstd", "snappy"])
@pytest.mark.parametrize("rows", [8000, 300_000])
def test_binary_dict_freq_general_exceptions(ctx, codec, rows):
    """A Dict whose index stream is Freq and whose exceptions stream is a
    general codec (binary/dict.rs:80-81 forbids only Dict below a Dict,
    integer/freq.rs:80-83 only Freq below a Freq): the exceptions expand into
    LDS (small page) or the page's region (big page), then scatter."""
    import pa_amd

    rng = np.random.default_rng(5)
    pool = [f"s{i:05d}".encode() for i in range(400)]
    s = [pool[0] if r < 0.95 else pool[int(x)] for r, x in zip(rng.random(rows), rng.integers(1, 400, rows))]
    dc = {"lz4": O.LZ4, "zstd": O.ZSTD, "snappy": O.SNAPPY}[codec]
    vals, offs = pa_amd.binary.strings_to_arrow(s)
    pg = O.write_binary_page(vals, offs, None, False, O.WriteOptions.make(ratio=2.0, forced=O.DICT, default_codec=dc),
                             offset_width=4, parent_values_len=len(vals))
    ib = 18
    bm = int.from_bytes(pg[ib + 4:ib + 8], "little")
    assert pg[0] == 11 and pg[9] == 13 and pg[ib + 8 + bm] == dc  # Dict -> Freq -> general exceptions
    check(ctx, s, None, False, rows, O.WriteOptions.make(ratio=2.0, forced=O.DICT, default_codec=dc), 13)


@pytest.mark.parametrize("page_rows", [1, 777, 8192])
def test_binary_ragged_pages(ctx, page_rows):
    rng = np.random.default_rng(4)
    n = 3000 if page_rows > 1 else 200
    s = strings("rand", n, rng)
    v = rng.random(n) > 0.3
    for opts in (O.WriteOptions.make(), O.WriteOptions.make(default_codec=O.LZ4), O.WriteOptions.make(ratio=2.0)):
        check(ctx, s, v, True, page_rows, opts, 13)
        check(ctx, s, None, False, page_rows, opts, 13)


@pytest.mark.parametrize("opt", ["plain", "dict", "freq", "adaptive", "zstd"])
def test_binary_two_pass_path(ctx, opt, monkeypatch):
    """The two-pass decode (k_bin_size -> k_bin_scan -> k_bin_decode) that a
    plan with header-only or big pages takes, forced on an all-staged column
    (SB_NO_BIN_FUSED): the same bytes as the fused pass."""
    monkeypatch.setenv("SB_NO_BIN_FUSED", "1")
    rng = np.random.default_rng(9)
    s = strings("freq" if opt == "freq" else "rand", 5000, rng)
    v = rng.random(5000) > 0.2
    assert check(ctx, s, v, True, 1000, O.WriteOptions.make(**OPTS[opt]), 13)
    assert check(ctx, s, None, False, 777, O.WriteOptions.make(**OPTS[opt]), 12)
