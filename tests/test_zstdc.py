"""The device encoder's Zstd frame writer (pa_amd/csrc/sb_zstdc.h), built for
the host, against the system libzstd: every frame decodes (ZSTD_decompress,
content size from the frame header) to the input bytes, and the oracle's Zstd
reader (the engine's decode path restated) agrees.  The reference writes
Zstd pages with zstd::bulk::compress level 0 (compression/basic.rs:122-135);
its bytes are not reproduced, decode equivalence is the bar (SURVEY.md
§8(f)1).  Inputs: the LZ4 compressor's edge set (tests/test_lz4c.py) plus
sizes on both sides of the 128 KiB chunk and 2048-sequence block limits.
No GPU needed."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests.test_lz4c import inputs

zstd = ctypes.CDLL("libzstd.so.1")
zstd.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
zstd.ZSTD_decompress.restype = ctypes.c_size_t
zstd.ZSTD_isError.argtypes = [ctypes.c_size_t]
zstd.ZSTD_isError.restype = ctypes.c_uint
zstd.ZSTD_getFrameContentSize.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
zstd.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong


def zbound(n):
    return n + n // 2048 + 3 * (n // 131072) + 512


def ours(data: bytes) -> bytes:
    import pa_amd

    L = pa_amd.lib()
    L.sb_zstd_compress_host.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.sb_zstd_compress_host.restype = ctypes.c_uint64
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    cap = zbound(len(data))
    dst = np.zeros(cap + 64, np.uint8)
    dst[cap:] = 0xA5
    r = L.sb_zstd_compress_host(src.ctypes.data, len(data), dst.ctypes.data)
    assert r <= cap and (dst[cap:] == 0xA5).all()
    return dst[:r].tobytes()


def libzstd_decode(frame: bytes) -> bytes:
    f = np.frombuffer(frame, np.uint8)
    n = zstd.ZSTD_getFrameContentSize(f.ctypes.data, len(frame))
    assert n < (1 << 62), "content size missing from the frame header"
    out = np.zeros(max(n, 1), np.uint8)
    r = zstd.ZSTD_decompress(out.ctypes.data, n, f.ctypes.data, len(frame))
    assert not zstd.ZSTD_isError(r), f"libzstd rejects the frame (code {r})"
    assert r == n
    return out[:n].tobytes()


def more_inputs():
    rng = np.random.default_rng(7)
    out = []
    for n in [131071, 131072, 131073, 262144 + 5, 600_000]:
        out.append(("small_alpha_chunks", rng.integers(0, 3, n, dtype=np.uint8).tobytes()))
    # many short sequences: > 2048 per chunk, so several compressed blocks
    out.append(("many_seqs", b"".join(bytes([i % 251, 7, 7, 7, 7, (i * 7) % 256]) for i in range(40000))))
    out.append(("f64_ints", rng.integers(0, 1000, 90000).astype(np.float64).tobytes()))
    out.append(("long_literals_then_match", rng.integers(0, 256, 70000, dtype=np.uint8).tobytes() + bytes(70000)))
    out.append(("huge_match", bytes(1_000_000)))
    return out


ALL = inputs() + more_inputs()


@pytest.mark.parametrize("case", range(len(ALL)))
def test_zstd_frame_decodes_with_libzstd(case):
    name, data = ALL[case]
    frame = ours(data)
    assert libzstd_decode(frame) == data, f"{name} n={len(data)}"
    assert O.common_decompress(O.ZSTD, frame, len(data)) == data


def test_zstd_frame_compresses():
    """Compressible pages shrink (the transcoded LZ4 parse, not Raw blocks)."""
    rng = np.random.default_rng(3)
    data = np.round(rng.standard_normal(20000) * 100, 1).astype(np.float64).tobytes()
    runs = np.repeat(rng.integers(0, 2**31, 300), 37).astype(np.int64).tobytes()
    for d in (bytes(100000), runs, bytes([1, 2, 3]) * 30000):
        assert len(ours(d)) < len(d) // 4
    assert len(ours(data)) < len(data)
