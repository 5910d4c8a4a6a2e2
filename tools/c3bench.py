"""Config-3 decoders timed separately (Float64 LZ4 nullable, Utf8 LZ4
nullable): python tools/c3bench.py [rows]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rng = np.random.default_rng(77)
    f = np.round(rng.standard_normal(rows) * 1e4, 2)
    fvalid = rng.random(rows) >= 0.1
    svals, soffs = bench.decimal_strings(rng.integers(0, 10**6, rows))
    svalid = rng.random(rows) >= 0.1
    opts = pa_amd.WriteOptions(default_compression=1, max_page_size=8192, seed=1)
    fchunk, fmetas = pa_amd.encode_column(f, fvalid, True, opts)
    schunk, smetas = pa_amd.encode_binary_column(svals, soffs, svalid, True, opts)
    print(f"f64: {len(fchunk)/rows/8:.3f} compressed/raw, utf8: {len(schunk)/(len(svals)+4*rows):.3f}")
    fd = pa_amd.ColumnDecoder(fchunk, fmetas, np.float64, True, timing=True)
    sd = pa_amd.BinaryColumnDecoder(schunk, smetas, pa_amd.UTF8, True, timing=True)
    fo, so = fd.alloc_outputs(), sd.alloc_outputs()
    for name, d, o, out_b in [("f64", fd, fo, rows * 8 + rows // 8), ("utf8", sd, so, 4 * rows + len(svals) + rows // 8)]:
        d.decode_async(*o)
        try:
            d.check()
        except Exception as e:  # timing-only variants (SB_INF_SKIP) decode garbage
            print(f"{name}: check failed: {e}")
        ts = []
        for _ in range(5):
            d.decode_async(*o)
            ts.append(d.last_kernel_ms())
        ms = float(np.median(ts))
        print(f"{name}: {ms:.3f} ms, {out_b / ms / 1e6:.1f} GB/s decoded", flush=True)


if __name__ == "__main__":
    main()
