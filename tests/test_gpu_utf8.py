"""UTF-8 validation of Utf8 / LargeUtf8 columns on the device.

The reference builds every Utf8 array with Utf8Array::try_new
(read/array/binary.rs:305-306), whose arrow2 0.17 check (restated in
oracle.check_utf8) rejects a values buffer that is not UTF-8 and an offset
inside a character.  The engine runs the same check after the decode
(k_utf8_bytes / k_utf8_bounds) and reports OutOfSpec for the page holding the
bad byte or row; a valid column decodes bit-exact against the oracle."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

POOL = ["a", "z", "0", " ", "é", "ß", "Ж", "ה", "€", "中", "文", "ｱ", "ࠀ", "￿", "퟿", "😀", "𝄞",
        "\U0010ffff", "\U00010000", "߿", "\u0080"]
# invalid sequences (RFC 3629): lone trail, overlong 2/3/4-byte, surrogate,
# above U+10FFFF, bytes that never appear, truncated 2/3/4-byte sequences
BAD = [b"\x80", b"\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xe0\x9f\xbf", b"\xf0\x80\x80\x80",
       b"\xf0\x8f\xbf\xbf", b"\xed\xa0\x80", b"\xed\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xfe",
       b"\xff", b"\xc3", b"\xe2\x82", b"\xf0\x9f\x98", b"\xc3\xa9\xa9", b"\xe2\x28\xa1"]


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def text(rng, n, maxlen=12):
    return [("".join(rng.choice(POOL, int(rng.integers(0, maxlen))))).encode() for _ in range(n)]


def encode(strs, nullable, opts, phys, rng, page_rows):
    import pa_amd

    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    valid = rng.random(len(strs)) > 0.2 if nullable else None
    o = pa_amd.WriteOptions(max_page_size=page_rows, **opts)
    return pa_amd.encode_binary_column(vals, offs, valid, nullable, o, physical_type=phys)


def status(ctx, dec):
    from pa_amd import _native as N

    dec.decode_async()
    bad = ctypes.c_int64(-1)
    st = N.lib().sb_plan_status(ctx._h, dec._h, ctypes.byref(bad))
    return st, bad.value


OPTS = {"plain": {}, "lz4": dict(default_compression=1), "zstd": dict(default_compression=2),
        "dict": dict(default_compress_ratio=2.0, forced_codec=11),
        "freq": dict(default_compress_ratio=2.0, forced_codec=13)}


@pytest.mark.parametrize("opt", list(OPTS))
@pytest.mark.parametrize("phys", ["UTF8", "LARGE_UTF8"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_valid_unicode_columns(ctx, opt, phys, nullable):
    """Multi-byte text across codecs decodes and passes the check, bit-exact."""
    import pa_amd

    rng = np.random.default_rng(5)
    n = 20_000
    pool = text(rng, 300) if opt in ("dict", "freq") else None
    strs = [pool[i] for i in rng.integers(0, 300, n)] if pool else text(rng, n)
    if opt == "freq":
        strs = [s if rng.random() < 0.05 else "共通の値".encode() for s in strs]
    pt = getattr(pa_amd, phys)
    chunk, metas = encode(strs, nullable, OPTS[opt], pt, rng, 4096)
    o, v, m = pa_amd.BinaryColumnDecoder(chunk, metas, pt, nullable, ctx).decode()
    eo, ev, em = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], nullable,
                                      offset_width=8 if phys == "LARGE_UTF8" else 4)
    assert O.check_utf8(ev, eo)
    assert (o.cpu().numpy() == eo).all()
    assert v.cpu().numpy()[:len(ev)].tobytes() == ev


@pytest.mark.parametrize("opt", ["plain", "lz4", "dict"])
@pytest.mark.parametrize("bad", range(len(BAD)))
def test_invalid_sequence_each_page_position(ctx, opt, bad):
    """One invalid sequence at the first, a middle and the last row of a page
    (and at byte offsets 0..15 of a 16-byte chunk): OutOfSpec on that page."""
    import pa_amd

    rng = np.random.default_rng(bad)
    page_rows, n = 500, 2000
    base = text(rng, n, 6)
    for row in (0, 499, 500, 1234, 1999):
        for pre in ((b"", b"abcdefghijklmno"[: row % 16]) if opt == "plain" else (b"",)):
            strs = list(base)
            strs[row] = pre + BAD[bad] + (b"x" if bad % 2 else b"")
            chunk, metas = encode(strs, False, OPTS[opt], pa_amd.UTF8, rng, page_rows)
            eo, ev, _ = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], False)
            assert not O.check_utf8(ev, eo)
            dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx)
            st, page = status(ctx, dec)
            assert st == pa_amd._native.E_OUT_OF_SPEC and page == row // page_rows, (row, st, page)
            dec.close()


def test_binary_type_accepts_any_bytes(ctx):
    """Binary / LargeBinary arrays are not checked (BinaryArray::try_new)."""
    import pa_amd

    rng = np.random.default_rng(1)
    strs = [bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(5000)]
    for pt in (pa_amd.BINARY, pa_amd.LARGE_BINARY):
        chunk, metas = encode(strs, False, {}, pt, rng, 1000)
        dec = pa_amd.BinaryColumnDecoder(chunk, metas, pt, False, ctx)
        assert status(ctx, dec) == (0, -1)
        dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8 if pt == pa_amd.BINARY else pa_amd.LARGE_UTF8,
                                         False, ctx)
        assert status(ctx, dec)[0] == pa_amd._native.E_OUT_OF_SPEC


@pytest.mark.parametrize("row", [1, 499, 500, 501, 1999])
def test_offset_inside_a_character(ctx, row):
    """The values buffer is valid UTF-8 but the offset starting `row` points at
    a trail byte ('é' split over two rows): OutOfSpec, as the reference's
    char-boundary check; rows at a page edge may be reported on either page."""
    import pa_amd

    rng = np.random.default_rng(row)
    strs = text(rng, 2000, 5)
    strs[row - 1] = strs[row - 1] + b"\xc3"
    strs[row] = b"\xa9" + strs[row]
    chunk, metas = encode(strs, False, {}, pa_amd.UTF8, rng, 500)
    eo, ev, _ = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], False)
    ev.decode("utf-8")  # the buffer itself is valid
    assert not O.check_utf8(ev, eo)
    st, page = status(ctx, pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx))
    assert st == pa_amd._native.E_OUT_OF_SPEC and page in {(row - 1) // 500, row // 500}, (st, page)


def test_fuzz_against_oracle(ctx):
    """Random mutations of random text (byte flips, inserts, splits): the
    device accepts a column exactly when oracle.check_utf8 does."""
    import pa_amd

    rng = np.random.default_rng(99)
    agree = {True: 0, False: 0}
    for case in range(300):
        n = int(rng.integers(1, 120))
        strs = text(rng, n, 20)
        for _ in range(int(rng.integers(0, 3))):
            i = int(rng.integers(0, n))
            s = bytearray(strs[i])
            op = int(rng.integers(0, 3))
            if op == 0 and s:
                s[int(rng.integers(0, len(s)))] = int(rng.integers(128, 256))
            elif op == 1:
                s.insert(int(rng.integers(0, len(s) + 1)), int(rng.integers(0, 256)))
            elif op == 2 and s and i + 1 < n:
                k = int(rng.integers(0, len(s)))
                strs[i + 1] = bytes(s[k:]) + strs[i + 1]
                del s[k:]
            strs[i] = bytes(s)
        chunk, metas = encode(strs, bool(case % 2), OPTS[["plain", "lz4", "dict"][case % 3]], pa_amd.UTF8, rng,
                              int(rng.integers(1, 64)))
        eo, ev, _ = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], bool(case % 2))
        want = O.check_utf8(ev, eo)
        dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, bool(case % 2), ctx)
        st, _ = status(ctx, dec)
        assert (st == 0) == want, (case, st, want)
        dec.close()
        agree[want] += 1
    assert agree[True] > 50 and agree[False] > 50, agree


def test_unaligned_values_buffer(ctx):
    """A values buffer that is not 16-byte aligned takes the byte-load path."""
    import pa_amd

    rng = np.random.default_rng(8)
    strs = text(rng, 3000)
    chunk, metas = encode(strs, False, {}, pa_amd.UTF8, rng, 1000)
    dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx)
    o, _, _ = dec.alloc_outputs()
    raw = torch.empty(dec.values_bytes + 32, dtype=torch.uint8, device="cuda")
    v = raw[3:3 + dec.values_bytes + 16]
    dec.decode_async(o, v, None)
    dec.check()
    eo, ev, _ = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], False)
    assert v.cpu().numpy()[:len(ev)].tobytes() == ev
    strs[2500] = b"ok\xffok"
    chunk, metas = encode(strs, False, {}, pa_amd.UTF8, rng, 1000)
    dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx)
    o, _, _ = dec.alloc_outputs()
    dec.decode_async(o, raw[5:5 + dec.values_bytes + 16], None)
    with pytest.raises(pa_amd.StrawboatError):
        dec.check()


@pytest.mark.parametrize("valid", [True, False])
def test_nested_utf8_leaf_checked(ctx, tmp_path, valid):
    """List<Utf8>: the leaf array is a Utf8Array too (read/array/binary.rs:288),
    so an invalid leaf string fails the column; valid text decodes."""
    import pa_amd

    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    from tests.test_pyarrow_nested import data_pages_v2, leaf_pages, utf8_stream

    rng = np.random.default_rng(3)
    rows = [[s for s in text(rng, int(rng.integers(0, 4)))] for _ in range(3000)]
    if not valid:
        rows[2100] = [b"ok", b"\xed\xa0\x80"]
    t = pa.table({"c": pa.array(rows, type=pa.list_(pa.binary()))})
    path = str(tmp_path / "u.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False, data_page_size=4096,
                   write_statistics=False)
    chunk, metas = leaf_pages(data_pages_v2(path, True), 3, 2, lambda sd, pl, e: utf8_stream(sd, pl, 3))
    dec = pa_amd.NestedColumnDecoder(chunk, [pa_amd.PageMeta(l, m) for l, m in metas], np.uint8, [True], True, ctx,
                                     physical_type=pa_amd.UTF8)
    if valid:
        dec.decode()
    else:
        with pytest.raises(pa_amd.StrawboatError) as e:
            dec.decode()
        assert e.value.status == pa_amd._native.E_OUT_OF_SPEC


def _dict_page_with_extra_entry(page: bytes, extra: bytes) -> bytes:
    """A non-nullable binary Dict page (binary/dict.rs:55-93 layout: [11]
    [csize][usize] [index stream] [u32 k] k x ([u64 len][bytes])) with one more
    dictionary entry that no row references."""
    assert page[0] == O.DICT
    body = page[9:]
    ic = int.from_bytes(body[1:5], "little")
    kpos = 9 + ic
    k = int.from_bytes(body[kpos:kpos + 4], "little")
    body = body[:kpos] + (k + 1).to_bytes(4, "little") + body[kpos + 4:] + len(extra).to_bytes(8, "little") + extra
    return bytes([O.DICT]) + len(body).to_bytes(4, "little") + page[5:9] + body


@pytest.mark.parametrize("opt", ["dict", "freq", "one"])
def test_extend_entries_checked_once(ctx, opt):
    """Dict / Freq / OneValue pages (the fused pass validates each entry once
    instead of the emitted rows): valid multi-byte entries decode; an invalid
    entry any row references -- a dictionary entry, the Freq top value or an
    exception, the OneValue -- is OutOfSpec on its page, as the reference's
    check of the emitted values buffer."""
    import pa_amd

    rng = np.random.default_rng(3)
    n, page_rows = 6000, 1500
    pool = text(rng, 40, 8) + ["€uro".encode(), "日本語テキスト".encode()]
    if opt == "one":
        strs = ["同じ値".encode()] * n
        o = dict(default_compress_ratio=2.0)
    elif opt == "freq":
        strs = [pool[i] if rng.random() < 0.05 else "共通の値".encode() for i in rng.integers(0, len(pool), n)]
        o = OPTS["freq"]
    else:
        strs = [pool[i] for i in rng.integers(0, len(pool), n)]
        o = OPTS["dict"]
    for nullable in (False, True):
        chunk, metas = encode(strs, nullable, o, pa_amd.UTF8, rng, page_rows)
        codecs = set(O.page_codec(chunk[sum(m.length for m in metas[:i]):], nullable) for i in range(len(metas)))
        assert codecs == {{"dict": O.DICT, "freq": O.FREQ, "one": O.ONE_VALUE}[opt]}, codecs
        dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, nullable, ctx)
        assert status(ctx, dec) == (0, -1)
        oo, v, _ = dec.decode()
        eo, ev, _ = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], nullable)
        assert (oo.cpu().numpy() == eo).all() and v.cpu().numpy()[:len(ev)].tobytes() == ev
        dec.close()
    for row in (0, 2999, 5999):
        bad = list(strs)
        if opt == "one":
            bad = [b"ab\xe2\x28\xa1"] * n if row == 0 else bad
            if row:
                continue
        elif opt == "freq" and row == 2999:  # the top value itself
            bad = [b"\xc3" if s == "共通の値".encode() else s for s in strs]
        else:
            bad[row] = b"x\xed\xa0\x80"
        chunk, metas = encode(bad, False, o, pa_amd.UTF8, rng, page_rows)
        eo, ev, _ = O.read_binary_column(chunk, [(x.length, x.num_values) for x in metas], False)
        assert not O.check_utf8(ev, eo)
        dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx)
        st, page = status(ctx, dec)
        assert st == pa_amd._native.E_OUT_OF_SPEC, (opt, row, st)
        if not (opt == "freq" and row == 2999):
            assert page == row // page_rows, (opt, row, page)
        dec.close()


def test_unreferenced_invalid_dict_entry_is_not_checked(ctx):
    """An invalid dictionary entry that no row references never reaches the
    values buffer, so Utf8Array::try_new accepts the array: the page's
    emitted bytes are then checked as they are, and pass."""
    import pa_amd

    rng = np.random.default_rng(4)
    pool = [f"v{i}é".encode() for i in range(20)]
    strs = [pool[i] for i in rng.integers(0, 20, 800)]
    chunk, metas = encode(strs, False, OPTS["dict"], pa_amd.UTF8, rng, 800)
    assert len(metas) == 1
    page = _dict_page_with_extra_entry(chunk, b"\xff\xfe")
    m = [pa_amd.PageMeta(len(page), 800)]
    eo, ev, _ = O.read_binary_column(page, [(len(page), 800)], False)
    assert O.check_utf8(ev, eo) and ev == b"".join(strs)
    dec = pa_amd.BinaryColumnDecoder(page, m, pa_amd.UTF8, False, ctx)
    assert status(ctx, dec) == (0, -1)
    oo, v, _ = dec.decode()
    assert (oo.cpu().numpy() == eo).all() and v.cpu().numpy()[:len(ev)].tobytes() == ev
