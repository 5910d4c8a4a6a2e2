"""Utf8 column decode time per C5 string kind: python tools/binbench.py [rows] [kind,kind...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
    rng = np.random.default_rng(5)
    kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["dict", "freq", "one", "lz4"]
    for kind in kinds:
        svals, soffs = bench.WorkloadC5._strings(kind, rows, rng)
        opts = pa_amd.WriteOptions(default_compression=1 if kind == "lz4" else 0,
                                   default_compress_ratio=None if kind == "lz4" else 2.0, max_page_size=8192, seed=3)
        chunk, metas = pa_amd.encode_binary_column(svals, soffs, None, False, opts, physical_type=pa_amd.UTF8, n_threads=16)
        mix = bench.page_codecs(chunk, metas, False)
        d = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False, timing=True)
        o = d.alloc_outputs()
        ts = []
        for _ in range(4):
            d.decode_async(*o)
            d.check()
            ts.append(d.last_kernel_ms())
        ms = float(np.median(ts[1:]))
        out_b = len(svals) + 4 * (rows + 1)
        print(f"{kind}: mix {mix} compressed {len(chunk)} {ms:.3f} ms, {out_b / ms / 1e6:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
