"""A C5-shaped Float64 Patas column (8.4M rows, 8192-row pages, the "patas"
value kind of bench.WorkloadC5) decoded alone: ms per decode (host clock,
median of 10) and bit-exactness against the source values:
python tools/patasbench.py [rows]  (SB_NO_PATAS_WG=1: the one-wave decoder)"""
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

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
    rng = np.random.default_rng(7)
    v = bench.WorkloadC5._values(np.float64, "patas", rows, rng)
    opts = pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=bench.PAGE_ROWS, forbidden_compressions=())
    chunk, metas = pa_amd.encode_column(v, None, False, opts, n_threads=16)
    mix = bench.page_codecs(chunk, metas, False)
    print("codecs", mix, "compressed", len(chunk), flush=True)
    dec = pa_amd.ColumnDecoder(torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda(), metas, np.float64, False)
    vals, _ = dec.decode()
    ok = vals.cpu().numpy().view(np.float64)[:rows].tobytes() == v.tobytes()
    ts = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dec.decode_async(vals, None)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dec.check()
    print(f"patas column: {np.median(ts) * 1e3:.3f} ms, bit-exact {ok}", flush=True)
    from pa_amd import _native as N
    L = N.lib()
    if hasattr(L, "sb_debug_pat_phases"):  # variant built with -DSB_PAT_PHASES (PA_AMD_LIB)
        import ctypes
        L.sb_debug_pat_reset()
        dec.decode_async(vals, None)
        torch.cuda.synchronize()
        buf = (ctypes.c_uint64 * 16)()
        L.sb_debug_pat_phases(buf)
        pages = max(1, buf[8])
        names = ["stage", "seg walks", "doubling+scan", "record starts", "terms", "jumping", "store"]
        print(f"pages {buf[8]} jumping rounds/page {buf[9] / pages:.1f}; shader cycles per page:",
              ", ".join(f"{k} {buf[i] / pages:.0f}" for i, k in enumerate(names)), flush=True)


if __name__ == "__main__":
    main()
