"""Malformed offsets in Basic LZ4 / Snappy Utf8 pages (header-only path:
offsets expanded and rebased by k_inflate, checked by k_bin_light_out).

  p[0] != 0   decompress_binary (binary/mod.rs:119-145) keeps the first
              page's p[0] as the column's offsets[0] and drops p[0] of every
              later page: no error, output equal to the oracle's.
  p[n] != S   DEVIATION: the device reports OutOfSpec for the page (the
              values base of the next page is the scan of the values
              lengths); the reference only fails if the column's last offset
              ends past its values (try_new in read_binary)."""
import ctypes

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


def page(codec, strs, fix=None):
    import pa_amd

    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    offs = offs.astype(np.int32)
    if fix:
        fix(offs)
    ob, vb = offs.tobytes(), vals
    oc, vc = O.common_compress(codec, ob), O.common_compress(codec, vb)
    hdr = lambda body, raw: bytes([codec]) + len(body).to_bytes(4, "little") + len(raw).to_bytes(4, "little")  # noqa: E731
    return hdr(oc, ob) + oc + hdr(vc, vb) + vc


def column(codec, bad_page, fix, rng):
    import pa_amd

    pages = []
    for i in range(3):
        strs = [str(x).encode() for x in rng.integers(0, 10**6, 3000)]
        pages.append(page(codec, strs, fix if i == bad_page else None))
    return b"".join(pages), [pa_amd.PageMeta(len(p), 3000) for p in pages]


@pytest.mark.parametrize("codec", [1, 3], ids=["lz4", "snappy"])
@pytest.mark.parametrize("bad_page", [0, 1])
def test_first_offset_not_zero(ctx, codec, bad_page):
    import pa_amd

    chunk, metas = column(codec, bad_page, lambda o: o.__setitem__(0, 5), np.random.default_rng(3))
    eo, ev, _ = O.read_binary_column(chunk, [(m.length, m.num_values) for m in metas], False)
    o, v, _ = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx).decode()
    assert (o.cpu().numpy() == eo).all()
    assert o[0].item() == (5 if bad_page == 0 else 0)
    assert v.cpu().numpy()[:len(ev)].tobytes() == ev


@pytest.mark.parametrize("codec", [1, 3], ids=["lz4", "snappy"])
@pytest.mark.parametrize("delta", [1, -1])
def test_last_offset_not_values_length(ctx, codec, delta):
    import pa_amd
    from pa_amd import _native as N

    chunk, metas = column(codec, 1, lambda o: o.__setitem__(len(o) - 1, o[-1] + delta), np.random.default_rng(4))
    dec = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx)
    dec.decode_async()
    badp = ctypes.c_int64(-1)
    st = N.lib().sb_plan_status(ctx._h, dec._h, ctypes.byref(badp))
    assert st == N.E_OUT_OF_SPEC and badp.value == 1, (st, badp.value, ctx.error())
