"""The multi-threaded CPU baseline driver (oracle/sb_cpu_mt.c) decodes exactly
what the single-threaded oracle readers decode, for any thread count and for
page sizes that put shard cuts on unaligned bitmap positions."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.colgen import build_column, gen_values


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("page_rows", [1000, 8192, 77])
def test_mt_flat(threads, page_rows):
    rng = np.random.default_rng(1)
    n = 50000
    for dtype, kind in [(np.int32, "index"), (np.float64, "full"), (np.int64, "runs")]:
        v = gen_values(kind, n, dtype, rng)
        valid = rng.random(n) > 0.2
        chunk, metas, _ = build_column(v, valid, True, page_rows, O.WriteOptions.make(ratio=1.2, default_codec=O.LZ4))
        ev, em = O.read_column(chunk, metas, dtype, True)
        gv, gm = O.mt_read_column(chunk, metas, dtype, True, threads)
        assert gv[:n].tobytes() == ev.tobytes()
        assert (np.unpackbits(gm, bitorder="little")[:n].astype(bool) == em).all()


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_mt_binary(threads):
    rng = np.random.default_rng(2)
    s = [str(x).encode() for x in rng.integers(0, 10**6, 30000)]
    vals, offs = O.strings_to_arrow(s)
    valid = rng.random(len(s)) > 0.1
    pages, metas = [], []
    for i in range(0, len(s), 999):
        m = min(999, len(s) - i)
        pg = O.write_binary_page(vals, offs[i:i + m + 1], valid[i:i + m], True, O.WriteOptions.make(default_codec=O.LZ4))
        pages.append(pg)
        metas.append((len(pg), m))
    chunk = b"".join(pages)
    eo, ev, em = O.read_binary_column(chunk, metas, True, 4)
    go, gv, gm, vl = O.mt_read_binary_column(chunk, metas, True, 4, threads, len(vals) + 16)
    assert vl == len(ev)
    assert (go.astype(np.int64) == eo).all()
    assert gv[:vl].tobytes() == ev
    assert (np.unpackbits(gm, bitorder="little")[:len(s)].astype(bool) == em).all()


@pytest.mark.parametrize("threads", [1, 5])
def test_mt_list_and_bool(threads):
    rng = np.random.default_rng(3)
    rows = 20000
    lens = rng.integers(0, 3, rows)
    lv = rng.random(rows) >= 0.1
    lens[~lv] = 0
    offs = np.zeros(rows + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    child = rng.integers(0, 1 << 16, int(offs[-1])).astype(np.int32)
    cv = rng.random(len(child)) >= 0.2
    chunk, metas, _ = O.write_list_column(offs, lv, child, cv, True, True, 1000, O.WriteOptions.make(ratio=1.2))
    eo, el, ev, ef = O.read_list_column(chunk, metas, np.int32, True, True)
    go, gl, gv, gf, r, v = O.mt_read_list_column(chunk, metas, np.int32, True, True, threads)
    assert (r, v) == (rows, len(child))
    assert (go[:rows + 1] == eo).all()
    assert gv[:v].tobytes() == ev.tobytes()
    assert (np.unpackbits(gl, bitorder="little")[:rows].astype(bool) == el).all()
    assert (np.unpackbits(gf, bitorder="little")[:v].astype(bool) == ef).all()

    b = np.repeat(rng.random(300) > 0.5, 100)
    bv = rng.random(len(b)) > 0.1
    pages, bm = [], []
    for i in range(0, len(b), 4096):
        m = min(4096, len(b) - i)
        pages.append(O.write_bool_page(b, bv[i:i + m], True, O.WriteOptions.make(ratio=1.2), offset=i, n=m))
        bm.append((len(pages[-1]), m))
    ch = b"".join(pages)
    evb, evm = O.read_bool_column(ch, bm, True)
    gvb, gvm = O.mt_read_bool_column(ch, bm, True, threads)
    assert (np.unpackbits(gvb, bitorder="little")[:len(b)].astype(bool) == evb).all()
    assert (np.unpackbits(gvm, bitorder="little")[:len(b)].astype(bool) == evm).all()
