"""Config-shaped parity at scale (BASELINE.json configs 2-5, SURVEY.md
§8(d) generators): each config's columns, at millions of rows, decoded on
the GPU through the C ABI and compared byte for byte with the oracle's read
of the same chunk -- values under null slots included, validity bitmaps,
offsets and list bitmaps.  (The small-page sweeps live in test_gpu_decode /
binary / list; bench.py checks the full-size configs against their source
values.)"""
import os
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (the generators)

THREADS = 16


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def _m(metas):
    return [(m.length, m.num_values) for m in metas]


def _bits(pa_amd, t, n):
    return pa_amd.read.unpack_bitmap(t, n).cpu().numpy()


def check_flat(pa_amd, ctx, v, valid, nullable, opts):
    chunk, metas = pa_amd.encode_column(v, valid, nullable, opts, n_threads=THREADS)
    got, gm = pa_amd.ColumnDecoder(chunk, metas, v.dtype, nullable, ctx).decode()
    ev, em = O.read_column(chunk, _m(metas), v.dtype, nullable)
    assert got.cpu().numpy()[:len(v)].tobytes() == ev.tobytes()  # values under nulls included
    if nullable:
        assert (_bits(pa_amd, gm, len(v)) == em).all()
    return chunk, metas


@pytest.mark.parametrize("variant", ["mix", "hard", "b12"])
def test_c2_20m_rows(ctx, variant):
    import pa_amd

    v = bench.gen_c2(20_000_000, 42, variant)
    chunk, metas = check_flat(pa_amd, ctx, v, None, False,
                              pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=8192))
    assert len(metas) == 2442


def test_c3_float64_lz4_nullable_5m(ctx):
    import pa_amd

    rng = np.random.default_rng(77)
    n = 5_000_000
    v = np.round(rng.normal(0, 1e4, n), 2)
    check_flat(pa_amd, ctx, v, rng.random(n) >= 0.1, True, pa_amd.WriteOptions(default_compression=1, max_page_size=8192))


def test_c3_utf8_lz4_nullable_5m(ctx):
    import pa_amd

    rng = np.random.default_rng(78)
    n = 5_000_000
    svals, soffs = bench.decimal_strings(rng.integers(0, 10**6, n))
    valid = rng.random(n) >= 0.1
    chunk, metas = pa_amd.encode_binary_column(svals, soffs, valid, True,
                                               pa_amd.WriteOptions(default_compression=1, max_page_size=8192),
                                               n_threads=THREADS)
    o, vals, m = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, True, ctx).decode()
    eo, ev, em = O.read_binary_column(chunk, _m(metas), True)
    assert (o.cpu().numpy() == eo).all()
    assert vals.cpu().numpy()[:len(ev)].tobytes() == ev
    assert (_bits(pa_amd, m, n) == em).all()


def test_c4_list_int32_5m(ctx):
    import pa_amd

    rng = np.random.default_rng(99)
    rows = 5_000_000
    lens = rng.integers(0, 3, rows)
    lv = rng.random(rows) >= 0.1
    lens[~lv] = 0
    offs = np.zeros(rows + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    child = rng.integers(0, 1 << 16, int(offs[-1])).astype(np.int32)
    cv = rng.random(len(child)) >= 0.2
    chunk, metas = pa_amd.encode_list_column(offs, child, lv, cv, True, True,
                                             pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=8192),
                                             n_threads=THREADS)
    go, glv, gv, gfv = pa_amd.ListColumnDecoder(chunk, metas, np.int32, True, True, ctx).decode()
    eo, elv, ev, efv = O.read_list_column(chunk, _m(metas), np.int32, True, True)
    V = len(child)
    assert (go.cpu().numpy().astype(np.int64) == eo).all()
    assert (_bits(pa_amd, glv, rows) == elv).all()
    assert gv.cpu().numpy()[:V].tobytes() == ev.tobytes()  # values under null items included
    assert (_bits(pa_amd, gfv, V) == efv).all()


C5_COLS = ([(np.int32, k) for k in dict.fromkeys(bench.WorkloadC5.I32)] +
           [(np.int64, k) for k in dict.fromkeys(bench.WorkloadC5.I64)] +
           [(np.float64, k) for k in dict.fromkeys(bench.WorkloadC5.F64)] +
           [(np.uint32, k) for k in dict.fromkeys(bench.WorkloadC5.U32)] +
           [(np.bool_, k) for k in dict.fromkeys(bench.WorkloadC5.BOOL)])


@pytest.mark.parametrize("dt,kind", C5_COLS, ids=[f"{np.dtype(d).name}-{k}" for d, k in C5_COLS])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_c5_column_1m(ctx, dt, kind, nullable):
    import pa_amd

    rng = np.random.default_rng(555)
    n = 1 << 20
    v = bench.WorkloadC5._values(dt, kind, n, rng)
    valid = rng.random(n) >= 0.1 if nullable else None
    plain = kind in ("lz4", "none")
    opts = (pa_amd.WriteOptions(default_compression=1 if kind == "lz4" else 0, max_page_size=8192) if plain else
            pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=8192))
    if dt == np.bool_:
        chunk, metas = pa_amd.encode_column(v, valid, nullable, opts, n_threads=THREADS)
        gv, gm = pa_amd.ColumnDecoder(chunk, metas, np.bool_, nullable, ctx).decode()
        ev, em = O.read_bool_column(chunk, _m(metas), nullable)
        assert (_bits(pa_amd, gv, n) == ev).all()
        if nullable:
            assert (_bits(pa_amd, gm, n) == em).all()
    else:
        check_flat(pa_amd, ctx, v, valid, nullable, opts)


@pytest.mark.parametrize("kind", list(dict.fromkeys(bench.WorkloadC5.STR)))
def test_c5_utf8_1m(ctx, kind):
    import pa_amd

    rng = np.random.default_rng(556)
    n = 1 << 20
    svals, soffs = bench.WorkloadC5._strings(kind, n, rng)
    opts = (pa_amd.WriteOptions(default_compression=1, max_page_size=8192) if kind == "lz4" else
            pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=8192))
    chunk, metas = pa_amd.encode_binary_column(svals, soffs, None, False, opts, n_threads=THREADS)
    o, vals, _ = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, ctx).decode()
    eo, ev, _ = O.read_binary_column(chunk, _m(metas), False)
    assert (o.cpu().numpy() == eo).all()
    assert vals.cpu().numpy()[:len(ev)].tobytes() == ev
