"""Phase breakdown of k_inflate's LZ4 batch loop (variant built with
-DSB_INF_PHASES, selected by PA_AMD_LIB): shader cycles per batch and per
sequence for the C3 Float64 and Utf8 columns.
python tools/infphases.py [rows]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["slide", "cand", "chain", "parse+place", "literals", "free", "hazards", "flush", "serial"]


def main():
    import torch

    import bench
    import pa_amd
    from pa_amd import _native as N

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rng = np.random.default_rng(77)
    f = np.round(rng.standard_normal(rows) * 1e4, 2)
    fvalid = rng.random(rows) >= 0.1
    svals, soffs = bench.decimal_strings(rng.integers(0, 10**6, rows))
    svalid = rng.random(rows) >= 0.1
    opts = pa_amd.WriteOptions(default_compression=1, max_page_size=8192, seed=1)
    fchunk, fmetas = pa_amd.encode_column(f, fvalid, True, opts)
    schunk, smetas = pa_amd.encode_binary_column(svals, soffs, svalid, True, opts)
    L = N.lib()
    buf = (ctypes.c_uint64 * 16)()
    for name, d in [("f64", pa_amd.ColumnDecoder(fchunk, fmetas, np.float64, True)),
                    ("utf8", pa_amd.BinaryColumnDecoder(schunk, smetas, pa_amd.UTF8, True))]:
        o = d.alloc_outputs()
        d.decode_async(*o)
        torch.cuda.synchronize()
        L.sb_debug_inf_reset()
        d.decode_async(*o)
        torch.cuda.synchronize()
        L.sb_debug_inf_phases(buf)
        a = np.frombuffer(buf, np.uint64).astype(np.float64)
        nb, ns, nh, nser, nj = a[9], a[10], a[11], a[12], a[13]
        tot = a[:9].sum()
        print(f"{name}: jobs {nj:.0f} batches {nb:.0f} seq/batch {ns / max(nb, 1):.1f} hazards/batch {nh / max(nb, 1):.1f} "
              f"serial seqs {nser:.0f}; cycles per batch {tot / max(nb, 1):.0f}, per job {tot / max(nj, 1):.0f}")
        print("  " + "  ".join(f"{p} {a[i] / max(nb, 1):.0f} ({100 * a[i] / tot:.0f}%)" for i, p in enumerate(PHASES)),
              flush=True)


if __name__ == "__main__":
    main()
