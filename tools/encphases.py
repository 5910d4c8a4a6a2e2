"""Per-page phase times of the device adaptive encode (variant built with
-DSB_ENC_PHASES): python tools/encphases.py [rows] -> median us per phase by
chosen codec, for the C2 column at ratio 1.2."""
import collections
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

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    v = bench.gen_c2(rows, 42, "mix")
    tv = torch.from_numpy(v).cuda()
    opts = pa_amd.WriteOptions(max_page_size=bench.PAGE_ROWS, default_compress_ratio=1.2, seed=42)
    for _ in range(2):
        pa_amd.encode_column_device(tv, None, False, opts)
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * (4096 * 12))()
    N.lib().sb_debug_enc_phases.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    N.lib().sb_debug_enc_phases(buf, 4096 * 12)
    a = np.frombuffer(buf, np.uint64).reshape(4096, 12).astype(np.int64)
    a = a[a[:, 0] > 0]
    span = (a[:, 3].max() - a[:, 0].min()) / 100.0  # s_memrealtime: 100 MHz -> us
    print(f"pages {len(a)} span {span:.1f} us", flush=True)
    by = collections.defaultdict(list)
    for i, (c0, c1) in enumerate(a[:, 8:10]):
        by[(int(c0), int(c1) if a[i, 4] > a[i, 2] else -1)].append(i)
    us = lambda x: float(np.median(x)) / 100.0
    for (c0, c1), ix in sorted(by.items()):
        b = a[ix]
        line = (f"codec {c0} (inner {c1}): {len(ix)} pages; median us stats {us(b[:, 1] - b[:, 0]):.1f} "
                f"choose {us(b[:, 2] - b[:, 1]):.1f} body {us(b[:, 3] - b[:, 2]):.1f}")
        if c1 >= 0:
            line += (f" [before inner {us(b[:, 4] - b[:, 2]):.1f}; inner stats {us(b[:, 5] - b[:, 4]):.1f} "
                     f"choose {us(b[:, 6] - b[:, 5]):.1f} body {us(b[:, 7] - b[:, 6]):.1f}; after {us(b[:, 3] - b[:, 7]):.1f}]")
        print(line, flush=True)


if __name__ == "__main__":
    main()
