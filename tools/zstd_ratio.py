"""Size of the device Zstd frame writer (sb_zstdc.h, run on the host through
sb_zstd_compress_host -- the same bytes the device writes) against libzstd
level 3 (the reference's zstd::bulk::compress level 0) on C3's two columns,
page by page (8192 rows): the Float64 values and the Utf8 page's two Basic
streams (rebased int32 offsets, value bytes).  CPU only:
python tools/zstd_ratio.py [pages]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import pa_amd
    from pa_amd import _native as N

    pages = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    rows = pages * 8192
    L = N.lib()
    L.sb_zstd_compress_host.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.sb_zstd_compress_host.restype = ctypes.c_uint64
    Z = ctypes.CDLL("libzstd.so.1")
    Z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    Z.ZSTD_compress.restype = ctypes.c_size_t
    Z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    Z.ZSTD_decompress.restype = ctypes.c_size_t

    def ours(b: bytes) -> int:
        dst = np.zeros(len(b) + len(b) // 2048 + 3 * (len(b) // 131072) + 512, np.uint8)
        n = L.sb_zstd_compress_host(b, len(b), dst.ctypes.data)
        back = np.zeros(max(len(b), 1), np.uint8)
        r = Z.ZSTD_decompress(back.ctypes.data, len(b), dst.ctypes.data, n)
        assert r == len(b) and back[:len(b)].tobytes() == b, "libzstd does not decode the frame to the input"
        return int(n)

    def lib3(b: bytes) -> int:
        dst = np.zeros(len(b) + 1024, np.uint8)
        return int(Z.ZSTD_compress(dst.ctypes.data, len(dst), b, len(b), 3))

    rng = np.random.default_rng(3)
    f = np.round(rng.standard_normal(rows) * 1e4, 2)
    svals, soffs = bench.decimal_strings(rng.integers(0, 10**6, rows))
    res = {}
    o = t = 0
    for p in range(pages):
        b = f[p * 8192:(p + 1) * 8192].tobytes()
        o += ours(b)
        t += lib3(b)
    res["c3_float64"] = (o, t)
    o = t = 0
    for p in range(pages):
        offs = soffs[p * 8192:(p + 1) * 8192 + 1]
        a = (offs - offs[0]).astype(np.int32).tobytes()
        v = svals[int(offs[0]):int(offs[-1])]
        o += ours(a) + ours(v)
        t += lib3(a) + lib3(v)
    res["c3_utf8"] = (o, t)
    for k, (o, t) in res.items():
        print(f"{k}: ours {o} libzstd3 {t} ratio {o / t:.3f}")


if __name__ == "__main__":
    main()
