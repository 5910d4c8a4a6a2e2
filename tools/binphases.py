"""Per-page phase times of the fused binary decode (variant built with
-DSB_BIN_PHASES): python tools/binphases.py [kind] -> median us per phase."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd
    from pa_amd import _native as N

    rows = 8 * 1024 * 1024
    rng = np.random.default_rng(5)
    for kind in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["dict", "freq", "one"]):
        svals, soffs = bench.WorkloadC5._strings(kind, rows, rng)
        opts = pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=8192, seed=3)
        chunk, metas = pa_amd.encode_binary_column(svals, soffs, None, False, opts, physical_type=pa_amd.UTF8, n_threads=16)
        d = pa_amd.BinaryColumnDecoder(chunk, metas, pa_amd.UTF8, False)
        o = d.alloc_outputs()
        for _ in range(3):
            d.decode_async(*o)
        d.check()
        torch.cuda.synchronize()
        buf = (ctypes.c_uint64 * (4096 * 6))()
        N.lib().sb_debug_bin_phases(buf, 4096 * 6)
        a = np.frombuffer(buf, np.uint64).reshape(4096, 6)[:len(metas), :5].astype(np.int64)
        dt = np.diff(a, axis=1) / 100.0  # s_memrealtime: 100 MHz -> us
        span = (a[:, 4].max() - a[:, 0].min()) / 100.0
        print(f"{kind}: pages {len(metas)} span {span:.1f} us; per page median us: stage+parse {np.median(dt[:, 0]):.1f} "
              f"tables {np.median(dt[:, 1]):.1f} lookback {np.median(dt[:, 2]):.1f} emit {np.median(dt[:, 3]):.1f}; "
              f"p90 lookback {np.percentile(dt[:, 2], 90):.1f}", flush=True)
        t0 = a[:, 0].min()
        st, en = (a[:, 0] - t0) / 100.0, (a[:, 4] - t0) / 100.0
        ev = sorted([(x, 1) for x in st] + [(x, -1) for x in en])
        cur = peak = 0
        for _, d_ in ev:
            cur += d_
            peak = max(peak, cur)
        tot = en - st
        print(f"    peak pages in flight {peak}; page total us mean {tot.mean():.1f} p10 {np.percentile(tot, 10):.1f} "
              f"p90 {np.percentile(tot, 90):.1f} max {tot.max():.1f}; starts at us: p50 {np.percentile(st, 50):.1f} "
              f"p90 {np.percentile(st, 90):.1f} last {st.max():.1f}; ends p50 {np.percentile(en, 50):.1f}", flush=True)


if __name__ == "__main__":
    main()
