"""ColumnGroupDecoder (sb_plan_column_at): several leaves of one type and
nullability, their chunks back to back, decoded as one plan -- each leaf's
views byte-identical to its own ColumnDecoder's arrays and to the oracle."""
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


def column(rng, dt, kind, n):
    if dt == np.bool_:
        return rng.random(n) > (0.5 if kind != "runs" else 0.0)
    if kind == "lz4":
        return np.round(rng.standard_normal(n) * 1e4, 2).astype(dt) if np.dtype(dt).kind == "f" else \
            rng.integers(0, 1 << 30, n).astype(dt)
    if kind == "runs":
        return np.repeat(rng.integers(0, 1000, n // 100 + 1), 100)[:n].astype(dt)
    return rng.integers(0, 5000, n).astype(dt)


@pytest.mark.parametrize("dt", [np.int32, np.int64, np.float64, np.uint16, np.bool_])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_group_equals_single(ctx, dt, nullable):
    import pa_amd

    rng = np.random.default_rng(7)
    kinds = ["plain", "lz4", "runs", "adaptive", "plain"]
    rows = [5000, 12345, 8192, 1, 40000]  # row counts not multiples of 32: the bases pad to 32
    cols, exp = [], []
    for kind, n in zip(kinds, rows):
        v = column(rng, dt, kind, n)
        valid = rng.random(n) > 0.15
        o = pa_amd.WriteOptions(default_compression=1 if kind == "lz4" else 0,
                                default_compress_ratio=2.0 if kind in ("adaptive", "runs") else None, max_page_size=1000)
        chunk, metas = pa_amd.encode_column(v, valid, nullable, o)
        cols.append((chunk, metas))
        exp.append(pa_amd.ColumnDecoder(chunk, metas, dt, nullable, ctx=ctx).decode())
    g = pa_amd.ColumnGroupDecoder(cols, dt, nullable, ctx=ctx)
    got = g.decode()
    for (gv, gm), (ev, em), (chunk, metas), n in zip(got, exp, cols, rows):
        if dt == np.bool_:
            nb = (n + 7) // 8
            assert gv.cpu().numpy()[:nb].tobytes()[:-1] == ev.cpu().numpy()[:nb].tobytes()[:-1]
            assert np.array_equal(np.unpackbits(gv.cpu().numpy(), bitorder="little")[:n],
                                  np.unpackbits(ev.cpu().numpy(), bitorder="little")[:n])
        else:
            assert gv.cpu().numpy().tobytes() == ev.cpu().numpy()[:n].tobytes()
            ov, _ = O.read_column(chunk, [(m.length, m.num_values) for m in metas], dt, nullable)
            assert gv.cpu().numpy().tobytes() == ov.tobytes()
        if nullable:
            assert np.array_equal(np.unpackbits(gm.cpu().numpy(), bitorder="little")[:n],
                                  np.unpackbits(em.cpu().numpy(), bitorder="little")[:n])
    g.close()


def test_group_rejects_overlapping_rows(ctx):
    import ctypes

    import pa_amd
    from pa_amd import _native as N

    v = np.arange(100, dtype=np.int32)
    chunk, metas = pa_amd.encode_column(v, None, False, pa_amd.WriteOptions(max_page_size=50))
    d = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda()
    cm = (N.PageMetaC * 2)(*[N.PageMetaC(m.length, m.num_values) for m in metas])
    ro = (ctypes.c_uint64 * 2)(0, 49)  # page 1 would overlap page 0's last row
    h = ctypes.c_void_p()
    st = N.lib().sb_plan_column_at(ctx._h, ctypes.byref(N.ColumnDescC(N.INT32, 0)), ctypes.c_void_p(d.data_ptr()),
                                   d.numel(), cm, 2, ro, ctypes.byref(h))
    assert st == N.E_ARG
