"""Device encode of Binary / Utf8 (sb_encode_binary_column_device) and
Boolean (sb_encode_column_device on a bitmap) columns against the oracle's
restatement of the writer, page by page (page p with sampler seed
page_seed(S, p)), and against the host writer's chunk:
  compress_binary   compression/binary/mod.rs:26-93 (OneValue / Freq / Dict,
                    Basic offsets + values streams; the Extend header's usize
                    is the parent array's values length)
  compress_boolean  compression/boolean/mod.rs:22-61 (forced RLE, OneValue /
                    RLE by ratio, Basic over the page's bitmap bytes)"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.colgen import same_pages_but_zstd

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

OPTS = {
    "plain": dict(ratio=None),
    "adaptive12": dict(ratio=1.2),
    "adaptive20": dict(ratio=2.0),
    "force_freq": dict(ratio=2.0, forced=O.FREQ),
    "force_dict": dict(ratio=2.0, forced=O.DICT),
    "force_rle": dict(ratio=2.0, forced=O.RLE),
    "lz4": dict(ratio=None, default_codec=O.LZ4),
    "lz4_adaptive": dict(ratio=1.2, default_codec=O.LZ4),
    "snappy": dict(ratio=None, default_codec=O.SNAPPY),
    "snappy_dict": dict(ratio=2.0, default_codec=O.SNAPPY, forced=O.DICT),
    "zstd": dict(ratio=None, default_codec=O.ZSTD),
    "tiny_ratio": dict(ratio=0.0001),
}


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def pa_opts(o, page_rows, seed=42):
    import pa_amd

    return pa_amd.WriteOptions(default_compression=o.get("default_codec", 0), default_compress_ratio=o.get("ratio"),
                               max_page_size=page_rows, forced_codec=o.get("forced", -1), seed=seed)


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
    if kind == "cat":
        return [f"category-{i:04d}".encode() for i in rng.integers(0, 200, n)]
    return [b"hello" if rng.random() < 0.95 else str(x).encode() for x in rng.integers(0, 1000, n)]


def check_binary(ctx, s, validity, nullable, page_rows, o, phys, seed=42):
    import pa_amd

    ow = 8 if phys in (pa_amd.LARGE_BINARY, pa_amd.LARGE_UTF8) else 4
    vals, offs = pa_amd.binary.strings_to_arrow(s)
    # a prefix of unreferenced bytes: offsets are absolute, parent_len is the whole buffer
    vals = b"PREFIX" + vals
    offs = offs + 6
    opts = pa_opts(o, page_rows, seed)
    tv = torch.from_numpy(np.frombuffer(vals, np.uint8).copy()).cuda()
    to = torch.from_numpy(offs.copy()).cuda()
    tvalid = torch.from_numpy(validity.copy()).cuda() if validity is not None else None
    dev, dm = pa_amd.encode_binary_column_device(tv, to, tvalid, nullable, opts, phys, ctx=ctx)
    got = dev.cpu().numpy().tobytes()
    host, hm = pa_amd.encode_binary_column(vals, offs, validity, nullable, opts, phys)
    if o.get("default_codec") == O.ZSTD:  # decode equivalence (same_pages_but_zstd)
        metas = same_pages_but_zstd(got, dm, host, hm, nullable)
        goffs, gvals, gvalid = O.read_binary_column(got, metas, nullable, offset_width=ow)
        for i in range(len(s)):
            if validity is None or not nullable or validity[i]:
                assert gvals[goffs[i]:goffs[i + 1]] == s[i], f"row {i}"
        return
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
    n = len(s)
    step = min(page_rows or n, n)
    pos = 0
    for p, i in enumerate(range(0, n, step)):
        m = min(step, n - i)
        oo = O.WriteOptions.make(seed=pa_amd.page_seed(seed, p), **o)
        exp = O.write_binary_page(vals, offs[i:i + m + 1], None if validity is None else validity[i:i + m], nullable,
                                  oo, offset_width=ow, parent_values_len=len(vals))
        assert got[pos:pos + len(exp)] == exp, f"page {p} differs"
        pos += len(exp)
    assert got == host


@pytest.mark.parametrize("opt", list(OPTS), ids=str)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
@pytest.mark.parametrize("phys", [13, 14], ids=["utf8", "large_utf8"])
def test_binary_columns(ctx, opt, nullable, phys):
    rng = np.random.default_rng(5)
    for kind in ["rand", "low", "one", "empty", "long", "cat", "freq"]:
        n = 5000
        s = strings(kind, n, rng)
        validity = (rng.random(n) > 0.2) if nullable else None
        for page_rows in (1024, 4096):
            check_binary(ctx, s, validity, nullable, page_rows, OPTS[opt], phys)


def test_binary_edges(ctx):
    """Mostly-null pages (Freq top_null), one-row pages, bitmap containers."""
    rng = np.random.default_rng(9)
    n = 10000
    s = strings("freq", n, rng)
    check_binary(ctx, s, rng.random(n) > 0.95, True, 8192, dict(ratio=1.0), 13)
    check_binary(ctx, s, rng.random(n) > 0.5, True, 1, dict(ratio=1.0, forced=O.DICT), 13)
    t = [b"a" if rng.random() < 0.5 else str(x).encode() for x in rng.integers(0, 50, 16384)]
    check_binary(ctx, t, None, False, 16384, dict(ratio=1.0, forced=O.FREQ), 13)


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


def check_bool(ctx, v, validity, nullable, page_rows, o, seed=42):
    import pa_amd

    opts = pa_opts(o, page_rows, seed)
    tv = torch.from_numpy(v.copy()).cuda()
    tvalid = torch.from_numpy(validity.copy()).cuda() if validity is not None else None
    dev, dm = pa_amd.encode_column_device(tv, tvalid, nullable, opts, ctx=ctx)
    got = dev.cpu().numpy().tobytes()
    host, hm = pa_amd.encode_column(v, validity, nullable, opts)
    if o.get("default_codec") == O.ZSTD:  # decode equivalence (same_pages_but_zstd)
        metas = same_pages_but_zstd(got, dm, host, hm, nullable)
        ov, _ = O.read_bool_column(got, metas, nullable)
        keep = validity if nullable else np.ones(len(v), bool)
        assert (np.asarray(ov)[:len(v)][keep] == v[keep]).all()
        return
    n = len(v)
    step = min(page_rows or n, n)
    pos = 0
    for p, i in enumerate(range(0, n, step)):
        m = min(step, n - i)
        oo = O.WriteOptions.make(seed=pa_amd.page_seed(seed, p), **o)
        exp = O.write_bool_page(v, None if validity is None or not nullable else validity[i:i + m], nullable, oo,
                                offset=i, n=m)
        assert got[pos:pos + len(exp)] == exp, f"page {p} differs"
        pos += len(exp)
    assert got == host
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]


@pytest.mark.parametrize("opt", list(OPTS), ids=str)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_bool_columns(ctx, opt, nullable):
    rng = np.random.default_rng(12)
    for kind in ["rand", "runs", "long_runs", "true", "false"]:
        for n, page_rows in ((20000, 8192), (5003, 1000), (700, 0), (9999, 13)):
            v = bool_values(kind, n, rng)
            validity = (rng.random(n) > 0.3) if nullable else None
            check_bool(ctx, v, validity, nullable, page_rows, OPTS[opt])
