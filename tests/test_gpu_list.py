"""GPU parity for nested List<primitive> columns: read_validity_nested
(read/read_basic.rs:65-173) + create_list (read/array/list.rs:48) + the
values streams, pages concatenated as batch_read_array does.  HIP path (C
ABI) vs the oracle, bit-exact: offsets, list validity, leaf values (bytes
under null items included) and leaf validity.  Pages from the oracle's
restatement of write_nested (serialize.rs:133-146, 217-232)."""
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


def make_lists(rows, rng, max_len=3, null_list=0.1, null_item=0.2, dtype=np.int32, vmax=1 << 16):
    """tests/it/io.rs:399-415 shape: lengths uniform in [0, max_len), null lists empty."""
    lens = rng.integers(0, max_len, rows)
    lv = rng.random(rows) >= null_list
    lens[~lv] = 0
    offs = np.zeros(rows + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    child = rng.integers(0, vmax, int(offs[-1])).astype(dtype)
    cv = rng.random(int(offs[-1])) >= null_item
    return offs, lv, child, cv


def gpu_list(ctx, chunk, metas, dtype, ln, inn, large=False):
    import pa_amd

    dec = pa_amd.ListColumnDecoder(chunk, [pa_amd.PageMeta(l, n) for l, n in metas], dtype, ln, inn, ctx, large=large)
    offs, lv, vals, fv = dec.decode()
    r, v = dec.num_rows, dec.num_leaves
    unpack = lambda b, n: np.unpackbits(b.cpu().numpy(), bitorder="little")[:n].astype(bool)  # noqa: E731
    out = (offs.cpu().numpy().astype(np.int64), unpack(lv, r) if ln else None,
           vals.cpu().numpy().view(np.uint8)[: v * np.dtype(dtype).itemsize].view(dtype), unpack(fv, v) if inn else None)
    dec.close()
    return out


def check(ctx, offs, lv, child, cv, ln, inn, page_rows, opts, large=False):
    chunk, metas, _ = O.write_list_column(offs, lv if ln else None, child, cv if inn else None, ln, inn, page_rows, opts)
    eo, el, ev, ef = O.read_list_column(chunk, metas, child.dtype, ln, inn)
    go, gl, gv, gf = gpu_list(ctx, chunk, metas, child.dtype, ln, inn, large)
    assert (go == eo).all(), "offsets differ"
    assert gv.tobytes() == ev.tobytes(), "values differ"
    if ln:
        assert (gl == el).all(), "list validity differs"
    if inn:
        assert (gf == ef).all(), "leaf validity differs"
    return chunk, metas


NEST = [(True, True), (False, False), (True, False), (False, True)]
OPTS = {
    "plain": dict(),
    "adaptive": dict(ratio=1.2),
    "adaptive2": dict(ratio=2.0),
    "lz4": dict(default_codec=O.LZ4),
    "zstd": dict(default_codec=O.ZSTD),
    "rle": dict(ratio=2.0, forced=O.RLE),
    "dict": dict(ratio=2.0, forced=O.DICT),
}


@pytest.mark.parametrize("nest", NEST, ids=["ln_in", "lr_ir", "ln_ir", "lr_in"])
@pytest.mark.parametrize("opt", list(OPTS))
@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float64, np.uint8], ids=lambda d: np.dtype(d).name)
def test_list_columns(ctx, nest, opt, dtype):
    rng = np.random.default_rng(21)
    ln, inn = nest
    offs, lv, child, cv = make_lists(30000, rng, dtype=dtype, vmax=200 if opt == "dict" else 1 << 16)
    check(ctx, offs, lv, child, cv, ln, inn, 8192, O.WriteOptions.make(seed=2, **OPTS[opt]))


@pytest.mark.parametrize("page_rows", [1, 7, 100, 1000, 0])
def test_list_ragged_pages(ctx, page_rows):
    rng = np.random.default_rng(page_rows)
    offs, lv, child, cv = make_lists(5000, rng)
    check(ctx, offs, lv, child, cv, True, True, page_rows, O.WriteOptions.make(ratio=1.2))


def test_list_repeated_decodes_multi_block(ctx):
    """k_list_bases tags each decode's block totals: one plan of 1 250 pages
    (five blocks exchanging totals) decoded again and again gives the
    oracle's arrays every time."""
    import pa_amd

    rng = np.random.default_rng(12)
    offs, lv, child, cv = make_lists(20000, rng)
    chunk, metas, _ = O.write_list_column(offs, lv, child, cv, True, True, 16, O.WriteOptions.make(ratio=1.2))
    eo, el, ev, ef = O.read_list_column(chunk, metas, child.dtype, True, True)
    dec = pa_amd.ListColumnDecoder(chunk, [pa_amd.PageMeta(l, n) for l, n in metas], np.int32, True, True, ctx)
    unpack = lambda b, n: np.unpackbits(b.cpu().numpy(), bitorder="little")[:n].astype(bool)  # noqa: E731
    for _ in range(5):
        go, gl, gv, gf = dec.decode()
        assert (go.cpu().numpy().astype(np.int64) == eo).all()
        assert (unpack(gl, dec.num_rows) == el).all() and (unpack(gf, dec.num_leaves) == ef).all()
        assert gv.cpu().numpy().view(np.uint8)[: 4 * dec.num_leaves].tobytes() == ev.tobytes()
    dec.close()


def test_list_9000_one_row_pages(ctx):
    """9 000 pages: k_list_bases' 36 workgroups exchange their totals, and
    k_list_levels walks more pages than it has waves."""
    rng = np.random.default_rng(9)
    offs, lv, child, cv = make_lists(9000, rng)
    check(ctx, offs, lv, child, cv, True, True, 1, O.WriteOptions.make())


def test_list_long_lists_multi_tile(ctx):
    """Pages with many levels per row: several level tiles per page; the
    level streams exceed the LDS stage and are read from HBM."""
    rng = np.random.default_rng(3)
    offs, lv, child, cv = make_lists(4000, rng, max_len=200)
    check(ctx, offs, lv, child, cv, True, True, 4000, O.WriteOptions.make())
    check(ctx, offs, lv, child, cv, False, True, 1500, O.WriteOptions.make(ratio=1.2))


def test_list_large_offsets_and_all_empty(ctx):
    rng = np.random.default_rng(4)
    offs, lv, child, cv = make_lists(3000, rng)
    check(ctx, offs, lv, child, cv, True, True, 700, O.WriteOptions.make(), large=True)
    offs0 = np.zeros(3001, np.int64)
    check(ctx, offs0, lv, child[:0], cv[:0], True, True, 700, O.WriteOptions.make())


def test_list_product_encoder_roundtrip(ctx):
    import pa_amd

    rng = np.random.default_rng(8)
    offs, lv, child, cv = make_lists(50000, rng)
    chunk, metas = pa_amd.encode_list_column(offs, child, lv, cv, True, True,
                                             pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=8192))
    go, gl, gv, gf = gpu_list(ctx, chunk, [(m.length, m.num_values) for m in metas], np.int32, True, True)
    assert (go == offs).all() and (gl == lv).all() and (gf == cv).all()
    assert (gv[cv] == child[cv]).all()


def test_list_hybrid_rle_runs(ctx):
    """Level streams with RLE runs (parquet writers other than arrow2 emit
    them; HybridRleDecoder reads both): rebuilt pages with the def stream as
    RLE + bit-packed runs must decode like the oracle."""
    rng = np.random.default_rng(5)
    rows = 600
    offs, lv, child, cv = make_lists(rows, rng, null_list=0.0, null_item=0.0)
    chunk, metas, _ = O.write_list_column(offs, None, child, None, False, False, 0, O.WriteOptions.make())
    L = metas[0][1]
    rep_len = int.from_bytes(chunk[4:8], "little")
    def_len = int.from_bytes(chunk[8:12], "little")
    # max_def = 1, bit width 1: every leaf level has def 1, empty lists 0
    defs = O.hybrid_decode(chunk[12 + rep_len:12 + rep_len + def_len], 1, L)
    k = 40
    assert (defs[:k] == defs[0]).all() or True
    # RLE run of the first k levels only when they are equal; else keep bit-packed
    first = int(defs[0])
    run = 1
    while run < L and defs[run] == first:
        run += 1
    rle = bytes([run << 1]) + bytes([first])
    rest = defs[run:]
    groups = (len(rest) + 7) // 8
    packed = np.packbits(np.concatenate([rest, np.zeros(groups * 8 - len(rest), np.uint32)]).astype(bool), bitorder="little")
    hdr = (groups << 1) | 1
    uleb = b""
    while True:
        c = hdr & 0x7F
        hdr >>= 7
        uleb += bytes([c | (0x80 if hdr else 0)])
        if not hdr:
            break
    new_def = rle + (uleb + packed.tobytes() if len(rest) else b"")
    page = chunk[:8] + len(new_def).to_bytes(4, "little") + chunk[12:12 + rep_len] + new_def + chunk[12 + rep_len + def_len:]
    m2 = [(len(page), L)]
    eo, _, ev, _ = O.read_list_column(page, m2, np.int32, False, False)
    go, _, gv, _ = gpu_list(ctx, page, m2, np.int32, False, False)
    assert (go == eo).all() and gv.tobytes() == ev.tobytes()


def test_list_malformed_pages(ctx):
    import pa_amd

    rng = np.random.default_rng(6)
    offs, lv, child, cv = make_lists(100, rng, null_list=0.0)
    chunk, metas, _ = O.write_list_column(offs, None, child, None, False, False, 0, O.WriteOptions.make())
    L = metas[0][1]
    cases = {
        "rows too many": (chunk[:0] + (101).to_bytes(4, "little") + chunk[4:], L),
        "short levels": (chunk[:12 + 1], L),
        "no rows": ((0).to_bytes(4, "little") + chunk[4:], L),
    }
    for name, (page, nl) in cases.items():
        with pytest.raises(pa_amd.StrawboatError):
            gpu_list(ctx, page, [(len(page), nl)], np.int32, False, False)
        with pytest.raises(O.OracleError):
            O.read_list_column(page, [(len(page), nl)], np.int32, False, False)


@pytest.mark.parametrize("dtype", [np.int32, np.float64, np.uint8], ids=lambda d: np.dtype(d).name)
def test_list_mixed_none_and_cascade_pages(ctx, dtype):
    """Pages whose values stream is None (the levels pass copies them and
    marks them done for the values plan) next to pages the values plan
    decodes (Dict, LZ4, Bitpacking), in one column, odd page sizes so the
    values start at every alignment."""
    rng = np.random.default_rng(31)
    opts = [O.WriteOptions.make(), O.WriteOptions.make(ratio=2.0, forced=O.DICT),
            O.WriteOptions.make(default_codec=O.LZ4), O.WriteOptions.make(ratio=2.0, forced=O.BITPACKING)]
    chunks, metas = [], []
    for k, op in enumerate(opts * 2):
        offs, lv, child, cv = make_lists(3000 + 37 * k, rng, dtype=dtype, vmax=200)
        if k % 4 == 3 and dtype == np.float64:
            op = O.WriteOptions.make()
        ch, me, _ = O.write_list_column(offs, lv, child, cv, True, True, 1001 + 2 * k, op)
        chunks.append(ch)
        metas += list(me)
    chunk = b"".join(chunks)
    eo, el, ev, ef = O.read_list_column(chunk, metas, np.dtype(dtype), True, True)
    go, gl, gv, gf = gpu_list(ctx, chunk, metas, np.dtype(dtype), True, True)
    assert (go == eo).all() and (gl == el).all() and (gf == ef).all()
    assert gv.tobytes() == ev.tobytes()
    # and decoded twice from one plan (the done marks are per decode)
    import pa_amd

    dec = pa_amd.ListColumnDecoder(chunk, [pa_amd.PageMeta(l, n) for l, n in metas], np.dtype(dtype), True, True, ctx)
    for _ in range(2):
        _, _, vals, _ = dec.decode()
        assert vals.cpu().numpy().view(np.uint8)[: len(ev) * np.dtype(dtype).itemsize].tobytes() == ev.tobytes()
    dec.close()
