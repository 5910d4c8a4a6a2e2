"""Patas leaf pages on the GPU (double/patas.rs:107-132): the workgroup-per-
page decoder (k_patas: segment walks for the record starts, pointer jumping
for the XOR references) against the oracle, for page sizes around its
segment and chunk edges, value shapes with every sig-byte count and
reference distance, pages too large for its LDS (k_inflate's one-wave
decoder takes those), and corrupted streams: the status must be the
oracle's code, the values bit-exact when the page decodes."""
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


def decode(ctx, pages, dtype, nullable=False):
    """-> (values, validity | None) or the StrawboatError status."""
    import pa_amd

    chunk = b"".join(p for p, _ in pages)
    dec = pa_amd.ColumnDecoder(np.frombuffer(chunk, np.uint8), [pa_amd.PageMeta(len(p), n) for p, n in pages],
                               dtype, nullable, ctx)
    try:
        v, bm = dec.decode()
    except pa_amd.StrawboatError as e:
        return e.status
    finally:
        dec.close()
    n = sum(k for _, k in pages)
    vals = v.cpu().numpy().view(np.uint8)[: n * np.dtype(dtype).itemsize].view(dtype)
    valid = np.unpackbits(bm.cpu().numpy(), bitorder="little")[:n].astype(bool) if nullable else None
    return vals, valid


def oracle(pages, dtype, nullable=False):
    try:
        return O.read_column(b"".join(p for p, _ in pages), [(len(p), n) for p, n in pages], dtype, nullable)
    except O.OracleError as e:
        return e.code


def shapes(rng, n, dtype):
    f32 = dtype == np.float32
    walk = (np.cumsum(rng.standard_normal(n)) * 10).astype(dtype)
    if f32:  # strictly increasing: no exact repeats in f32 (the reference's repeat desync, DESIGN deviation 2)
        walk = np.cumsum(np.abs(rng.standard_normal(n)) * 10 + 0.5).astype(dtype)
    out = {"walk": walk, "ramp": np.arange(n, dtype=dtype) * dtype(0.25)}
    if not f32:  # exact repeats: references up to 127 rows back (f32 repeats desync, DESIGN deviation 2)
        rep = walk.copy()
        rep[::3] = rep[0]
        out["repeats"] = rep
        out["pool"] = rng.choice(rng.standard_normal(40), n).astype(dtype)
        out["const"] = np.full(n, 1.5, dtype)
        sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-300, 1.5], dtype)
        out["special"] = sp[rng.integers(0, len(sp), n)]
    out["noise"] = rng.standard_normal(n).astype(dtype)
    return out


def patas_page(v, validity=None, nullable=False):
    page = O.write_page(v, validity, nullable, O.WriteOptions.make(ratio=1.0, forced=O.PATAS))
    assert O.page_codec(page, nullable) == O.PATAS
    return page


@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("n", [1, 2, 3, 64, 65, 129, 255, 256, 257, 1000, 4096, 4097, 8192, 12000, 16384, 24000])
def test_patas_pages_match_oracle(ctx, dtype, n):
    rng = np.random.default_rng(n)
    for name, v in shapes(rng, n, dtype).items():
        page = patas_page(v)
        exp = oracle([(page, n)], dtype)
        got = decode(ctx, [(page, n)], dtype)
        assert not isinstance(exp, int), name
        assert not isinstance(got, int), (name, got)
        assert got[0].tobytes() == exp[0].tobytes(), name


@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=lambda d: np.dtype(d).name)
def test_patas_columns_many_pages(ctx, dtype):
    """Pages of 8192 rows (C5's shape) and ragged ones in one column, with and
    without validity, several workgroups' worth of pages."""
    rng = np.random.default_rng(5)
    for nullable in (False, True):
        pages, total = [], 0
        for k in range(40):
            n = 8192 if k % 3 else int(rng.integers(1, 9000))
            v = shapes(rng, n, dtype)["walk" if k % 2 else ("repeats" if dtype == np.float64 else "ramp")]
            valid = rng.random(n) > 0.1 if nullable else None
            pages.append((patas_page(v, valid, nullable), n))
            total += n
        exp = oracle(pages, dtype, nullable)
        got = decode(ctx, pages, dtype, nullable)
        assert got[0].tobytes() == exp[0].tobytes()
        if nullable:
            assert (got[1] == exp[1]).all()


def _body(page):
    assert page[0] == O.PATAS
    return bytearray(page[9:])


def _page(body, usize):
    return bytes([O.PATAS]) + len(body).to_bytes(4, "little") + usize.to_bytes(4, "little") + bytes(body)


@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=lambda d: np.dtype(d).name)
def test_corrupt_patas_pages_match_oracle(ctx, dtype):
    """Truncated streams (Io), references before row 0 (OutOfSpec), f32
    records with more than 4 sig bytes (OutOfSpec), trailing bytes (fine)
    and random byte flips: the device's status is the oracle's, and a page
    both accept decodes to the same values."""
    rng = np.random.default_rng(9)
    w = np.dtype(dtype).itemsize
    seen = {"ok": 0, "err": 0}
    for case in range(160):
        n = [3, 64, 200, 2000, 8192][case % 5]
        v = shapes(rng, n, dtype)["walk" if case % 2 else "ramp"]
        body = _body(patas_page(v))
        kind = case % 8
        if kind == 0:  # truncated
            body = body[: int(rng.integers(0, len(body)))]
        elif kind == 1:  # trailing bytes
            body += bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))
        elif kind == 2 and len(body) > w + 2:  # a header's ref_diff past row 0: patch the first record
            h = int.from_bytes(body[w:w + 2], "little")
            body[w:w + 2] = ((h & 0x1FF) | (int(rng.integers(2, 128)) << 9)).to_bytes(2, "little")
        elif kind == 3 and dtype == np.float32 and len(body) > w + 2:  # 5..7 sig bytes in an f32 record
            h = int.from_bytes(body[w:w + 2], "little")
            body[w:w + 2] = ((h & ~(7 << 6)) | (int(rng.integers(5, 8)) << 6) | 1).to_bytes(2, "little")
        else:
            for _ in range(int(rng.integers(1, 4))):
                if body:
                    i = int(rng.integers(0, len(body)))
                    body[i] ^= 1 << int(rng.integers(0, 8))
        page = _page(body, n * w)
        exp = oracle([(page, n)], dtype)
        got = decode(ctx, [(page, n)], dtype)
        if isinstance(exp, int):
            assert isinstance(got, int) and got == exp, (case, kind, got, exp)
            seen["err"] += 1
        else:
            assert not isinstance(got, int), (case, kind, got)
            assert got[0].tobytes() == exp[0].tobytes(), (case, kind)
            seen["ok"] += 1
    assert seen["ok"] > 20 and seen["err"] > 20, seen
