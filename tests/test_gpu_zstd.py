"""GPU parity for Zstd pages: CommonCompression::Zstd (compression/basic.rs:
93-97, 122-135; libzstd 1.4.8 through the zstd 0.11 crate) decoded by the
one-wave device frame decoder (pa_amd/csrc/sb_zstd.h) vs the oracle's
ZSTD_decompress, bit-exact, through the C ABI.

Frames: the writer's ZSTD_compress (level 3: single segment, content size,
one block per page) at every cascade position the Basic codec reaches, and --
for the multi-block paths a page-sized ZSTD_compress frame never takes
(Treeless literals, Repeat / RLE sequence tables, raw and RLE blocks, a window
descriptor, no content size) -- libzstd's streaming API with a flush every
few KiB at levels -5..19.  Bit-flipped frames must be rejected exactly when
libzstd rejects them and decode to libzstd's bytes otherwise."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests.colgen import build_column, gen_values, oracle_decode_column

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def gpu_decode(ctx, chunk, metas, dtype, nullable=False):
    import pa_amd

    dec = pa_amd.ColumnDecoder(chunk, [pa_amd.PageMeta(l, n) for l, n in metas], dtype, nullable, ctx)
    try:
        vals, bm = dec.decode()
        n = dec.num_rows
        v = vals.cpu().numpy().view(np.uint8)[: n * np.dtype(dtype).itemsize].view(dtype)
        m = np.unpackbits(bm.cpu().numpy(), bitorder="little")[:n].astype(bool) if nullable else None
        return v, m
    finally:
        dec.close()


class _ZBuf(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("size", ctypes.c_size_t), ("pos", ctypes.c_size_t)]


_Z = []


def _zlib():
    if not _Z:
        z = ctypes.CDLL("libzstd.so.1")
        z.ZSTD_createCCtx.restype = ctypes.c_void_p
        z.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
        z.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        z.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
        z.ZSTD_CCtx_setPledgedSrcSize.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
        z.ZSTD_CCtx_setPledgedSrcSize.restype = ctypes.c_size_t
        z.ZSTD_compressStream2.argtypes = [ctypes.c_void_p, ctypes.POINTER(_ZBuf), ctypes.POINTER(_ZBuf), ctypes.c_int]
        z.ZSTD_compressStream2.restype = ctypes.c_size_t
        z.ZSTD_isError.argtypes = [ctypes.c_size_t]
        z.ZSTD_isError.restype = ctypes.c_uint
        _Z.append(z)
    return _Z[0]


def stream_frame(data: bytes, pieces: int, level: int = 3, checksum: bool = False, pledged: bool = False) -> bytes:
    """One frame from libzstd's streaming API (ZSTD_compressStream2), flushed
    after each of `pieces` slices: every flush closes a block."""
    z = _zlib()
    cc = z.ZSTD_createCCtx()
    try:
        assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cc, 100, level))  # ZSTD_c_compressionLevel
        if checksum:
            assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cc, 201, 1))  # ZSTD_c_checksumFlag
        if pledged:
            assert not z.ZSTD_isError(z.ZSTD_CCtx_setPledgedSrcSize(cc, len(data)))
        src = ctypes.create_string_buffer(data, max(len(data), 1))
        out = ctypes.create_string_buffer(2 * len(data) + 4096)
        ob = _ZBuf(ctypes.addressof(out), len(out), 0)
        cuts = np.linspace(0, len(data), pieces + 1).astype(int)
        for i in range(pieces):
            ib = _ZBuf(ctypes.addressof(src) + int(cuts[i]), int(cuts[i + 1] - cuts[i]), 0)
            mode = 2 if i == pieces - 1 else 1  # ZSTD_e_end : ZSTD_e_flush
            while True:
                r = z.ZSTD_compressStream2(cc, ctypes.byref(ob), ctypes.byref(ib), mode)
                assert not z.ZSTD_isError(r)
                if r == 0 and ib.pos == ib.size:
                    break
        return out.raw[: ob.pos]
    finally:
        z.ZSTD_freeCCtx(cc)


def zstd_page(values: np.ndarray, frame: bytes) -> bytes:
    """A non-nullable Basic page [codec 2][csize][usize][frame] (the header
    compress_integer writes, compression/integer/mod.rs:35-70)."""
    return bytes([O.ZSTD]) + len(frame).to_bytes(4, "little") + values.nbytes.to_bytes(4, "little") + frame


def shapes(rng, n):
    idx = gen_values("index", n, np.int64, rng, uniq=300)
    full = gen_values("full", n, np.int64, rng)
    digits = "".join(str(x) for x in rng.integers(0, 10**6, n)).encode()
    return {
        "index": idx,
        "full": full,  # incompressible: raw blocks / raw literals
        "zeros": np.zeros(n, np.int64),  # RLE blocks / RLE literals / long matches
        "sorted": np.cumsum(rng.integers(0, 50, n)).astype(np.int64),
        "runs": gen_values("runs", n, np.int64, rng),
        "text": np.frombuffer((digits * 2)[: 8 * n], np.int64).copy(),
        "mixed": np.concatenate([full[: n // 2], idx[n // 2:]]),
    }


def check_page(ctx, values, page):
    n = len(values)
    ov, _ = O.read_page(page, n, values.dtype, False)
    assert ov.tobytes() == values.tobytes(), "oracle round trip"
    gv, _ = gpu_decode(ctx, page, [(len(page), n)], values.dtype)
    assert gv.tobytes() == ov.tobytes(), "device bytes differ from libzstd"


ZOPTS = {
    "plain": dict(default_codec=O.ZSTD),
    "adaptive12": dict(default_codec=O.ZSTD, ratio=1.2),
    "adaptive20": dict(default_codec=O.ZSTD, ratio=2.0),
    "dict": dict(default_codec=O.ZSTD, ratio=2.0, forced=O.DICT),
    "freq": dict(default_codec=O.ZSTD, ratio=2.0, forced=O.FREQ),
}


@pytest.mark.parametrize("dtype", [np.int32, np.int64, np.uint8, np.float32, np.float64], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("opt", list(ZOPTS))
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_writer_zstd_columns(ctx, dtype, opt, nullable):
    """The writer's frames: value leaves, Dict index streams, Freq exception
    streams, with and without validity."""
    rng = np.random.default_rng(17)
    for kind in ["index", "full", "one", "runs", "freq", "sorted"]:
        n = 20000
        v = gen_values(kind, n, dtype, rng)
        validity = (rng.random(n) > 0.2) if nullable else None
        opts = O.WriteOptions.make(forbidden=(O.PATAS,), **ZOPTS[opt])
        for page_rows in (1000, 8192):
            chunk, metas, _ = build_column(v, validity, nullable, page_rows, opts)
            ov, om = oracle_decode_column(chunk, metas, v.dtype, nullable)
            gv, gm = gpu_decode(ctx, chunk, metas, v.dtype, nullable)
            assert gv.tobytes() == ov.tobytes(), f"{kind}/{page_rows}: values differ"
            if nullable:
                assert (gm == om).all(), f"{kind}/{page_rows}: validity differs"


@pytest.mark.parametrize("level", [-5, 1, 3, 19])
@pytest.mark.parametrize("pieces", [1, 3, 9])
def test_stream_frames(ctx, level, pieces):
    """Multi-block frames: raw / RLE / compressed blocks, Treeless literals,
    Repeat and RLE sequence tables, with and without a content size."""
    rng = np.random.default_rng(1000 + 10 * pieces + level)
    for v in shapes(rng, 8192).values():
        for pledged in (False, True):
            check_page(ctx, v, zstd_page(v, stream_frame(v.tobytes(), pieces, level, pledged=pledged)))


def test_small_and_odd_sizes(ctx):
    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 33, 100, 1000, 4097):
        v = gen_values("index", n, np.int64, rng, uniq=20)
        for pieces in (1, 2):
            check_page(ctx, v, zstd_page(v, stream_frame(v.tobytes(), min(pieces, n), 3, pledged=True)))


def test_checksum_frames(ctx):
    """Frames with a content checksum (XXH64, low 32 bits) decode; a wrong
    checksum is rejected by both libzstd (the oracle) and the device."""
    import pa_amd

    rng = np.random.default_rng(8)
    for n in (3, 4, 5, 100, 4096, 20000):
        v = gen_values("index", n, np.int64, rng, uniq=97)
        for pieces in (1, 3):
            frame = stream_frame(v.tobytes(), min(pieces, n), 3, checksum=True, pledged=bool(pieces == 1))
            check_page(ctx, v, zstd_page(v, frame))
            bad = bytearray(frame)
            bad[-1 - int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 8))  # inside the 4 checksum bytes
            page = zstd_page(v, bytes(bad))
            with pytest.raises(O.OracleError):
                O.read_page(page, n, np.int64, False)
            with pytest.raises(pa_amd.StrawboatError):
                gpu_decode(ctx, page, [(len(page), n)], np.int64)


def skippable(payload: bytes, k: int = 0) -> bytes:
    """A skippable frame (RFC 8878 3.1.2): magic 0x184D2A50 + k, size, payload."""
    return (0x184D2A50 + k).to_bytes(4, "little") + len(payload).to_bytes(4, "little") + payload


def test_multiple_and_skippable_frames(ctx):
    """Several frames back to back, with skippable frames between them (as
    ZSTD_decompress, compression/basic.rs:93-97, accepts): the output is the
    frames' contents in order."""
    rng = np.random.default_rng(9)
    for n in (7, 1000, 9000):
        v = gen_values("runs", n, np.int64, rng)
        raw = v.tobytes()
        cuts = sorted({0, len(raw), *(int(x) for x in rng.integers(0, len(raw), 2))})
        parts = [raw[a:b] for a, b in zip(cuts, cuts[1:]) if b > a]
        for variant in range(4):
            frame = b""
            for k, part in enumerate(parts):
                if variant & 1:
                    frame += skippable(bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)), k)
                frame += stream_frame(part, 1 + (k % 2), 3, checksum=bool(variant & 2), pledged=bool(k % 2 == 0))
            if variant == 3:
                frame += skippable(b"tail", 15)
            check_page(ctx, v, zstd_page(v, frame))


def test_corrupt_frames_match_libzstd(ctx):
    """Bit flips anywhere in the frame: the device rejects exactly the frames
    libzstd rejects and decodes the others to libzstd's bytes."""
    import pa_amd

    rng = np.random.default_rng(99)
    base = [gen_values("index", 2048, np.int64, rng, uniq=300), np.cumsum(rng.integers(0, 9, 2048)).astype(np.int64)]
    seen = {"ok": 0, "err": 0}
    for t in range(240):
        v = base[t % 2]
        frame = bytearray(stream_frame(v.tobytes(), 1 + t % 3, 3, pledged=bool(t % 4)))
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, len(frame)))
            frame[i] ^= 1 << int(rng.integers(0, 8))
        page = zstd_page(v, bytes(frame))
        try:
            ov, _ = O.read_page(page, len(v), np.int64, False)
        except O.OracleError:
            ov = None
        gv, gst = None, 0
        try:
            gv, _ = gpu_decode(ctx, page, [(len(page), len(v))], np.int64)
        except pa_amd.StrawboatError as e:
            gst = e.status
        if ov is None:
            assert gv is None, f"case {t}: libzstd rejects the frame, the device decodes it"
            seen["err"] += 1
        else:
            assert gv is not None, f"case {t}: libzstd decodes the frame, the device reports status {gst}"
            assert gv.tobytes() == ov.tobytes(), f"case {t}: bytes differ"
            seen["ok"] += 1
    assert seen["ok"] and seen["err"]


def prefix_frame(data: bytes, prefix: bytes, level: int = 3) -> bytes:
    """A frame compressed against a referenced prefix (ZSTD_CCtx_refPrefix +
    ZSTD_compress2): its sequences reach back into the prefix, i.e. before
    the frame's own first output byte; no dictionary id is recorded."""
    z = _zlib()
    z.ZSTD_CCtx_refPrefix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    z.ZSTD_CCtx_refPrefix.restype = ctypes.c_size_t
    z.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    z.ZSTD_compress2.restype = ctypes.c_size_t
    cc = z.ZSTD_createCCtx()
    try:
        assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cc, 100, level))
        pre = ctypes.create_string_buffer(prefix, max(len(prefix), 1))
        assert not z.ZSTD_isError(z.ZSTD_CCtx_refPrefix(cc, pre, len(prefix)))
        out = ctypes.create_string_buffer(2 * len(data) + 4096)
        r = z.ZSTD_compress2(cc, out, len(out), data, len(data))
        assert not z.ZSTD_isError(r)
        return out.raw[:r]
    finally:
        z.ZSTD_freeCCtx(cc)


@pytest.mark.parametrize("n", [1000, 4096, 20000], ids=lambda n: f"rows{n}")
def test_match_into_previous_frame_is_rejected(ctx, n):
    """libzstd starts each frame's history at the frame's first output byte
    (ZSTD_checkContinuity per frame), so a second frame whose match reaches
    into the first frame's output is corrupt for ZSTD_decompress
    (compression/basic.rs:93-97) even though the bytes it would copy are
    right there: the device must reject it too.  20000 rows of Int64 is a
    page past the LDS stage (k_zinflate, HBM to HBM)."""
    import pa_amd

    rng = np.random.default_rng(n)
    a = gen_values("index", n // 2, np.int64, rng, uniq=1 << 20)
    raw = a.tobytes()
    second = prefix_frame(raw, raw)
    assert len(second) < len(raw) // 4, "the frame should be matches into the prefix"
    v = np.concatenate([a, a])
    page = zstd_page(v, stream_frame(raw, 1, 3, pledged=True) + second)
    with pytest.raises(O.OracleError):
        O.read_page(page, len(v), np.int64, False)
    with pytest.raises(pa_amd.StrawboatError):
        gpu_decode(ctx, page, [(len(page), len(v))], np.int64)
    # two self-contained frames of the same bytes decode
    ok = zstd_page(v, stream_frame(raw, 1, 3, pledged=True) + stream_frame(raw, 1, 3, pledged=True))
    check_page(ctx, v, ok)
