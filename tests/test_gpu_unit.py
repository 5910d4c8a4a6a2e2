"""Page-level unit entry points (sb_decode_page_validity,
sb_decode_page_levels): one flat page's validity prefix (read_validity,
read/read_basic.rs:36-63) and one nested page's rep / def level streams
(read_validity_nested, :65-86), bit-exact against the oracle's read_validity
and hybrid_decode, the level streams from the oracle's writer (one bit-packed
run) and from pyarrow's Data Page V2 pages (RLE and bit-packed runs)."""
import itertools

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


def bits_of(t, n, off=0):
    b = np.unpackbits(t.cpu().numpy().view(np.uint8), bitorder="little")
    return b[off:off + n].astype(bool)


@pytest.mark.parametrize("n", [1, 7, 8, 31, 32, 33, 1000, 8192, 100_003])
@pytest.mark.parametrize("bit_offset", [0, 5, 31, 32, 77])
def test_page_validity(ctx, n, bit_offset):
    from pa_amd.read import read_validity

    rng = np.random.default_rng(n + bit_offset)
    v = rng.integers(0, 1000, n).astype(np.int32)
    valid = rng.random(n) > 0.3
    page = O.write_page(v, valid, True)
    exp, pos = O.read_validity(page, n)
    # the bitmap's other bits are kept: start from all ones
    out = torch.full(((bit_offset + n + 31) // 32 + 1,), -1, dtype=torch.int32, device="cuda")
    got, used = read_validity(page, n, out, bit_offset, ctx=ctx)
    assert used == pos
    assert (bits_of(got, n, bit_offset) == exp).all()
    allb = np.unpackbits(got.cpu().numpy().view(np.uint8), bitorder="little").astype(bool)
    assert allb[:bit_offset].all() and allb[bit_offset + n:].all()


def test_page_validity_errors(ctx):
    import pa_amd
    from pa_amd.read import read_validity

    page = O.write_page(np.arange(100, dtype=np.int32), np.ones(100, bool), True)
    cases = {
        "rle run": (4).to_bytes(4, "little") + bytes([100 << 1, 1, 0, 0]),  # an RLE header: unreachable!()
        "short run": (3).to_bytes(4, "little") + bytes([(2 << 1) | 1, 0xFF, 0xFF]),  # 16 bits for 100 rows
        "truncated": page[:8],
        "def_len 0": (0).to_bytes(4, "little") + page[4:],
    }
    for name, pg in cases.items():
        with pytest.raises(pa_amd.StrawboatError) as e:
            read_validity(pg, 100, ctx=ctx)
        assert e.value.status in (pa_amd._native.E_OUT_OF_SPEC, pa_amd._native.E_IO), name
    # def_len 0 with no rows: nothing pushed, nothing wrong
    _, used = read_validity((0).to_bytes(4, "little"), 0, ctx=ctx)
    assert used == 4


@pytest.mark.parametrize("ln,inn", list(itertools.product([False, True], repeat=2)))
def test_page_levels_oracle_writer(ctx, ln, inn):
    from pa_amd.read import read_levels

    rng = np.random.default_rng(3 + 2 * ln + inn)
    rows = 5000
    lens = rng.integers(0, 6, rows)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    lv = rng.random(rows) > 0.1
    child = rng.integers(0, 1 << 20, int(offs[-1])).astype(np.int32)
    cv = rng.random(len(child)) > 0.2
    chunk, metas, prow = O.write_list_column(offs, lv if ln else None, child, cv if inn else None, ln, inn, 1000)
    max_def = int(ln) + 1 + int(inn)
    pos = 0
    for (length, nlev), r in zip(metas, prow):
        page = chunk[pos:pos + length]
        pos += length
        rl = int.from_bytes(page[4:8], "little")
        dl = int.from_bytes(page[8:12], "little")
        erep = O.hybrid_decode(page[12:12 + rl], 1, nlev)
        edef = O.hybrid_decode(page[12 + rl:12 + rl + dl], max_def.bit_length(), nlev)
        rep, dfl, grows, used = read_levels(page, nlev, 1, max_def, ctx=ctx)
        assert grows == r and used == 12 + rl + dl
        assert (rep.cpu().numpy().astype(np.uint32) == erep).all()
        assert (dfl.cpu().numpy().astype(np.uint32) == edef).all()


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_page_levels_pyarrow_runs(ctx, tmp_path, depth):
    """pyarrow's level streams mix RLE and bit-packed runs (bit widths 1..3)."""
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    from pa_amd.read import read_levels
    from tests.test_pyarrow_nested import data_pages_v2

    rng = np.random.default_rng(depth)

    def build(level):
        r = rng.random()
        if r < 0.1:
            return None
        if r < 0.3:
            return []
        if level == depth - 1:
            return [None if rng.random() < 0.1 else int(x) for x in rng.integers(0, 9, int(rng.integers(1, 40)))]
        return [build(level + 1) for _ in range(int(rng.integers(1, 4)))]

    t = pa.table({"c": [build(0) for _ in range(4000)]})
    path = str(tmp_path / "l.parquet")
    pq.write_table(t, path, data_page_version="2.0", compression="NONE", use_dictionary=False, data_page_size=8192,
                   write_statistics=False)
    max_rep, max_def = depth, 2 * depth + 1
    for rows, nlev, rep_b, def_b, _ in data_pages_v2(path):
        page = rows.to_bytes(4, "little") + len(rep_b).to_bytes(4, "little") + len(def_b).to_bytes(4, "little")
        page += rep_b + def_b + b"\0" * 16
        rep, dfl, grows, used = read_levels(page, nlev, max_rep, max_def, ctx=ctx)
        assert grows == rows and used == 12 + len(rep_b) + len(def_b)
        assert (rep.cpu().numpy().astype(np.uint32) == O.hybrid_decode(rep_b, max_rep.bit_length(), nlev)).all()
        assert (dfl.cpu().numpy().astype(np.uint32) == O.hybrid_decode(def_b, max_def.bit_length(), nlev)).all()
