"""Config-5 decode units timed alone (median of 5 solo decodes, host clock
around decode + device synchronize), then the 4-stream step:
python tools/c5units.py [rows].  Each unit's solo decodes are separated by
10 ms of idle device, so a kernel trace of this run splits into units by its
gaps (tools/unit_kernels.py); the encode comes first."""
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
    wl = bench.WorkloadC5(torch, pa_amd, rows, 555, 0, 16)
    print(f"encode {wl.encode_gpu_s * 1e3:.1f} ms ({wl.raw_bytes / wl.encode_gpu_s / 1e9:.1f} GB/s)", flush=True)
    tot = 0.0
    for u in wl.units:
        dec, outs = u[0], u[1]
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            time.sleep(0.01)
            t0 = time.perf_counter()
            dec.decode_async(*outs)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ms = float(np.median(ts[1:]))
        tot += ms
        kind = type(dec).__name__
        cols = [ci for ci, c in enumerate(wl.cols) if c[1] is dec]
        what = sorted({(str(wl.cols[ci][0]) if not isinstance(wl.cols[ci][0], str) else "utf8") for ci in cols})
        print(f"{kind:20s} cols {cols} {what} {ms:.3f} ms", flush=True)
    print(f"sum of solo units {tot:.3f} ms", flush=True)
    w, k, ok = bench.timed(torch, None, wl, 10, 3)
    print(f"c5 step: {w / 10 * 1e3:.3f} ms, ok={ok}", flush=True)


if __name__ == "__main__":
    main()
