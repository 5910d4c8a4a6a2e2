"""Device List<primitive> encode (sb_encode_list_column_device) against the
host writer (sb_encode_list_column, itself byte-identical to the oracle's
write_list_column): encode_chunk + slice_parquet_array per page of top-level
rows (write/common.rs:49-119) and write_nested (serialize.rs:133-146) -- the
rep / def level streams (one bit-packed hybrid run each, the last chunk's
spare bits from the writer's reused buffer) and the sliced child values
through the cascade.  Bytes must be identical; the chunk must decode
(ListColumnDecoder) to the source lists."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def make_lists(rows, rng, max_len=3, null_list=0.1, null_item=0.2, dtype=np.int32, vmax=1 << 16):
    lens = rng.integers(0, max_len, rows)
    lv = rng.random(rows) >= null_list
    lens[~lv] = 0
    offs = np.zeros(rows + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    child = rng.integers(0, vmax, int(offs[-1])).astype(dtype)
    cv = rng.random(int(offs[-1])) >= null_item
    return offs, lv, child, cv


def both(ctx, offs, lv, child, cv, ln, inn, opts):
    import pa_amd

    hc, hm = pa_amd.encode_list_column(offs, child, lv if ln else None, cv if inn else None, ln, inn, opts)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    dc, dm = pa_amd.encode_list_column_device(dev(offs), dev(child), dev(lv) if ln else None, dev(cv) if inn else None,
                                              ln, inn, opts, ctx)
    return bytes(hc), hm, bytes(dc.cpu().numpy()), dm


def check(ctx, offs, lv, child, cv, ln, inn, opts):
    hc, hm, dc, dm = both(ctx, offs, lv, child, cv, ln, inn, opts)
    assert [(m.length, m.num_values) for m in dm] == [(m.length, m.num_values) for m in hm]
    assert dc == hc
    return dc, dm


NEST = [(True, True), (False, False), (True, False), (False, True)]


def opts_for(name, page):
    import pa_amd as pa
    from pa_amd.write import DICT, LZ4, RLE

    return {
        "plain": pa.WriteOptions(max_page_size=page),
        "adaptive": pa.WriteOptions(default_compress_ratio=1.2, max_page_size=page, seed=3),
        "adaptive2": pa.WriteOptions(default_compress_ratio=2.0, max_page_size=page, seed=4),
        "lz4": pa.WriteOptions(default_compression=LZ4, max_page_size=page),
        "dict": pa.WriteOptions(default_compress_ratio=2.0, forced_codec=DICT, max_page_size=page, seed=5),
        "rle": pa.WriteOptions(default_compress_ratio=2.0, forced_codec=RLE, max_page_size=page, seed=6),
    }[name]


@pytest.mark.parametrize("nest", NEST, ids=["ln_in", "lr_ir", "ln_ir", "lr_in"])
@pytest.mark.parametrize("opt", ["plain", "adaptive", "adaptive2", "lz4", "dict", "rle"])
@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.float64, np.uint8], ids=lambda d: np.dtype(d).name)
def test_device_list_encode_matches_host(ctx, nest, opt, dtype):
    rng = np.random.default_rng(41)
    ln, inn = nest
    offs, lv, child, cv = make_lists(20000, rng, dtype=dtype, vmax=200 if opt == "dict" else 1 << 16)
    check(ctx, offs, lv, child, cv, ln, inn, opts_for(opt, 8192))


@pytest.mark.parametrize("page", [1, 7, 31, 32, 33, 100, 1000])
def test_device_list_encode_ragged_pages(ctx, page):
    """Page sizes around the 32-level chunks (the spare bits of the last
    chunk come from the previous one) and the 8-level groups."""
    rng = np.random.default_rng(page)
    offs, lv, child, cv = make_lists(3000, rng)
    check(ctx, offs, lv, child, cv, True, True, opts_for("adaptive", page))
    check(ctx, offs, lv, child, cv, False, True, opts_for("plain", page))


def test_device_list_encode_long_and_empty(ctx):
    rng = np.random.default_rng(7)
    offs, lv, child, cv = make_lists(2000, rng, max_len=300)
    check(ctx, offs, lv, child, cv, True, True, opts_for("adaptive", 500))
    offs0 = np.zeros(3001, np.int64)  # every list empty: one level a row, no child values
    lv0 = rng.random(3000) >= 0.1
    check(ctx, offs0, lv0, np.zeros(0, np.int32), np.zeros(0, bool), True, True, opts_for("plain", 700))


def test_device_list_encode_decodes(ctx):
    """The device chunk decodes (ListColumnDecoder) to the source lists."""
    import pa_amd

    rng = np.random.default_rng(9)
    offs, lv, child, cv = make_lists(30000, rng)
    dc, dm = check(ctx, offs, lv, child, cv, True, True, opts_for("adaptive", 8192))
    dec = pa_amd.ListColumnDecoder(np.frombuffer(dc, np.uint8), [pa_amd.PageMeta(m.length, m.num_values) for m in dm],
                                   np.int32, True, True, ctx)
    go, gl, gv, gf = dec.decode()
    unpack = lambda b, n: np.unpackbits(b.cpu().numpy(), bitorder="little")[:n].astype(bool)  # noqa: E731
    assert (go.cpu().numpy().astype(np.int64) == offs).all()
    assert (unpack(gl, len(lv)) == lv).all()
    assert (unpack(gf, len(cv)) == cv).all()
    vals = gv.cpu().numpy().view(np.int32)[: len(child)]
    assert (vals[cv] == child[cv]).all()
    dec.close()


def test_device_list_encode_largest_page_step(ctx):
    """The largest page step the device List encoder takes (16384 rows):
    k_enc_list_levels' row-prefix table is 65540 B of dynamic LDS, past
    64 KiB."""
    rng = np.random.default_rng(16384)
    offs, lv, child, cv = make_lists(40000, rng)
    check(ctx, offs, lv, child, cv, True, True, opts_for("adaptive", 16384))
    check(ctx, offs, lv, child, cv, False, False, opts_for("lz4", 16384))


def test_device_list_encode_refuses_decreasing_offsets(ctx):
    """A decreasing offset pair -- at a page boundary or inside a page -- is an
    argument error, as in the host writer, not a wrapped slot size."""
    import pa_amd

    rng = np.random.default_rng(3)
    offs, lv, child, cv = make_lists(3000, rng)
    for at in (1000, 1234):  # page boundary (page 1000) and inside a page
        bad = offs.copy()
        bad[at] = bad[at + 1] + 1
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
        with pytest.raises(pa_amd.StrawboatError) as e:
            pa_amd.encode_list_column_device(dev(bad), dev(child), dev(lv), dev(cv), True, True,
                                             opts_for("plain", 1000), ctx)
        assert e.value.status == 6
