"""The one-shot C-ABI entry points, called through ctypes against the oracle:
sb_decode_column (plan + decode + wait + status in one call: the
batch_read_array shape for one flat leaf) and sb_decompress_values
(decompress_integer / decompress_double of ONE value stream with no validity
prefix: compression/integer/mod.rs:72-117, compression/double/mod.rs:69-114)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests.colgen import build_column, gen_values

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


@pytest.mark.parametrize("dtype", [np.int32, np.uint64, np.float64, np.int8], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_sb_decode_column(ctx, dtype, nullable):
    import pa_amd
    from pa_amd import _native as N

    rng = np.random.default_rng(4)
    n = 30000
    for kind, opts in (("index", O.WriteOptions.make(ratio=1.2)), ("runs", O.WriteOptions.make(ratio=2.0)),
                       ("full", O.WriteOptions.make(default_codec=O.LZ4))):
        v = gen_values(kind, n, dtype, rng)
        valid = rng.random(n) > 0.2 if nullable else None
        chunk, metas, _ = build_column(v, valid, nullable, 4096, opts)
        ev, em = O.read_column(chunk, metas, dtype, nullable)
        d_chunk = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda()
        out_v = torch.empty(n * np.dtype(dtype).itemsize, dtype=torch.uint8, device="cuda")
        out_m = torch.zeros(((n + 31) // 32) * 4, dtype=torch.uint8, device="cuda") if nullable else None
        pm = (N.PageMetaC * len(metas))(*[N.PageMetaC(l, m) for l, m in metas])
        desc = N.ColumnDescC(pa_amd.read.physical_type(dtype), int(nullable))
        out = N.PrimitiveOutC(out_v.data_ptr(), out_m.data_ptr() if nullable else None)
        st = N.lib().sb_decode_column(ctx._h, ctypes.byref(desc), ctypes.c_void_p(d_chunk.data_ptr()), len(chunk), pm,
                                      len(metas), ctypes.byref(out))
        assert st == 0, ctx.error()
        assert out_v.cpu().numpy().tobytes() == ev.view(np.uint8).tobytes()
        if nullable:
            assert (np.unpackbits(out_m.cpu().numpy(), bitorder="little")[:n].astype(bool) == em).all()
    # a malformed page: the status, not a crash
    bad = bytearray(chunk)
    bad[(4 + int.from_bytes(bad[:4], "little")) if nullable else 0] = 99
    d_bad = torch.from_numpy(np.frombuffer(bytes(bad), np.uint8).copy()).cuda()
    st = N.lib().sb_decode_column(ctx._h, ctypes.byref(desc), ctypes.c_void_p(d_bad.data_ptr()), len(bad), pm,
                                  len(metas), ctypes.byref(out))
    assert st == N.E_OUT_OF_SPEC


@pytest.mark.parametrize("dtype", [np.int32, np.uint32, np.int64, np.float32, np.float64, np.uint16],
                         ids=lambda d: np.dtype(d).name)
def test_sb_decompress_values(ctx, dtype):
    from pa_amd import _native as N

    rng = np.random.default_rng(6)
    for kind in ("index", "sorted", "one", "runs", "freq", "full"):
        # (Patas forbidden: an f32 stream with repeats is the reference's undecodable desync page)
        for o in (O.WriteOptions.make(ratio=1.2, forbidden=(O.PATAS,)), O.WriteOptions.make(ratio=2.0, forced=O.DICT),
                  O.WriteOptions.make(default_codec=O.SNAPPY), O.WriteOptions.make(ratio=2.0, forced=O.FREQ)):
            v = gen_values(kind, 8192, dtype, rng)
            stream = O.compress(v, None, o)
            ev, _ = O.decompress(stream, dtype, len(v))
            d = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).cuda()
            out = torch.empty(len(v) * np.dtype(dtype).itemsize, dtype=torch.uint8, device="cuda")
            st = N.lib().sb_decompress_values(ctx._h, __import__("pa_amd").read.physical_type(dtype),
                                              ctypes.c_void_p(d.data_ptr()), len(stream), len(v),
                                              ctypes.c_void_p(out.data_ptr()))
            assert st == 0, ctx.error()
            assert out.cpu().numpy().tobytes() == ev.tobytes()
