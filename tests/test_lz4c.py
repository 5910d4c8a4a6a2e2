"""The device encoder's block compressors (pa_amd/csrc/sb_lz4c.h), built for
the host, against the libraries whose bytes they must reproduce:
  * LZ4: the system liblz4 1.9.3 LZ4_compress_default (basic.rs:115 through
    the lz4 1.23 crate) -- byte for byte, over inputs on both sides of the
    64 KiB table switch (LZ4_64Klimit = 65547), the MFLIMIT / LASTLITERALS
    edges, long literal runs and long matches;
  * Snappy: the oracle's raw-snappy writer (oracle/sb_oracle.c), which the
    host writer matches.
No GPU needed."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

lz4 = ctypes.CDLL("liblz4.so.1")
lz4.LZ4_compress_default.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
lz4.LZ4_compress_default.restype = ctypes.c_int


def _lib():
    import pa_amd

    L = pa_amd.lib()
    for f in ("sb_lz4_compress_host", "sb_snappy_compress_host"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        getattr(L, f).restype = ctypes.c_uint64
    return L


def liblz4(data: bytes) -> bytes:
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    cap = len(data) + len(data) // 255 + 16
    dst = np.zeros(cap, np.uint8)
    r = lz4.LZ4_compress_default(src.ctypes.data, dst.ctypes.data, len(data), cap)
    assert r > 0
    return dst[:r].tobytes()


def ours(fn, data: bytes, cap: int) -> bytes:
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    dst = np.zeros(cap, np.uint8)
    r = getattr(_lib(), fn)(src.ctypes.data, len(data), dst.ctypes.data)
    assert r <= cap
    return dst[:r].tobytes()


def inputs():
    rng = np.random.default_rng(1)
    out = []
    for n in [0, 1, 4, 11, 12, 13, 14, 17, 64, 100, 1000, 4096, 65535, 65546, 65547, 65548, 70000, 200000, 300001]:
        out.append(("random", rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
        out.append(("zeros", bytes(n)))
        out.append(("small_alpha", rng.integers(0, 4, n, dtype=np.uint8).tobytes()))
    # strawboat page shapes: f64 values, decimal strings, offsets, runs, repeating patterns
    f = np.round(rng.standard_normal(8192) * 1e4, 2)
    out.append(("f64_page", f.tobytes()))
    out.append(("f64_big", np.round(rng.standard_normal(40000) * 1e4, 2).tobytes()))
    s = b"".join(str(x).encode() for x in rng.integers(0, 10**6, 8192))
    out.append(("decimal_strings", s))
    out.append(("offsets", np.cumsum(rng.integers(1, 7, 8193)).astype(np.int32).tobytes()))
    out.append(("runs", np.repeat(rng.integers(0, 2**31, 300), 37).astype(np.int64).tobytes()))
    out.append(("period3", bytes([1, 2, 3]) * 30000))
    out.append(("long_match_then_literals", bytes(5000) + rng.integers(0, 256, 3000, dtype=np.uint8).tobytes() + bytes(700)))
    out.append(("far_repeat", (rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()) * 2))
    return out


@pytest.mark.parametrize("case", range(len(inputs())))
def test_lz4_matches_liblz4(case):
    name, data = inputs()[case]
    got = ours("sb_lz4_compress_host", data, len(data) + len(data) // 255 + 16)
    assert got == liblz4(data), f"{name} n={len(data)}"


@pytest.mark.parametrize("case", range(len(inputs())))
def test_snappy_matches_writer(case):
    name, data = inputs()[case]
    got = ours("sb_snappy_compress_host", data, len(data) + len(data) // 20 + 32)
    assert got == O.common_compress(O.SNAPPY, data), f"{name} n={len(data)}"
    assert O.common_decompress(O.SNAPPY, got, len(data)) == data
