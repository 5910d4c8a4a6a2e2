"""Decode time of single C5-shaped fixed-width columns per value kind:
python tools/kindbench.py [rows] [dtype:kind,...]  (default: the Int64 and
Float64 kinds of bench.WorkloadC5).  Prints kernel ms (HIP events), decoded
GB/s and the page codec mix."""
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
    specs = (sys.argv[2].split(",") if len(sys.argv) > 2 else
             ["int64:runs", "int64:dict", "int64:freq", "int64:none", "int32:bp12", "int32:sorted",
              "float64:slow", "float64:patas", "float64:dict", "float64:runs", "float64:lz4", "uint32:bp18"])
    for sp in specs:
        dt, kind = sp.split(":")
        dt = np.dtype(dt)
        rng = np.random.default_rng(7)
        v = bench.WorkloadC5._values(dt.type, kind, rows, rng)
        basic = kind in ("lz4", "none")
        opts = pa_amd.WriteOptions(default_compression=1 if kind == "lz4" else 0,
                                   default_compress_ratio=None if basic else 2.0, max_page_size=8192, seed=5)
        chunk, metas = pa_amd.encode_column(v, None, False, opts, n_threads=16)
        d = pa_amd.ColumnDecoder(chunk, metas, dt, False, timing=True)
        o = d.alloc_outputs()
        ts = []
        for _ in range(6):
            d.decode_async(*o)
            d.check()
            ts.append(d.last_kernel_ms())
        ms = float(np.median(ts[1:]))
        ok = o[0].cpu().numpy().view(dt)[:rows].tobytes() == v.tobytes()
        mix = bench.page_codecs(chunk, metas, False)
        print(f"{sp:14s} {ms:7.3f} ms {v.nbytes / ms / 1e6:7.1f} GB/s out, {len(chunk) / ms / 1e6:7.1f} GB/s in, "
              f"ok={ok} mix {mix}", flush=True)


if __name__ == "__main__":
    main()
