"""Config-4 (List<Int32>) decode timed alone, kernel by kernel under rocprof:
python tools/c4bench.py [rows]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    pa_amd.default_context(0)
    wl = bench.WorkloadC4(torch, pa_amd, rows, 99, 0, 16)
    if os.environ.get("SB_NOCHECK"):  # timing-only variants whose output is knowingly wrong
        wl.verify = lambda torch: False
        for d in wl.decs:
            d.check = lambda: None
    print(f"pages {len(wl.metas)} leaves {wl.leaves} in {wl.in_bytes} out {wl.out_bytes}", flush=True)
    wall, k, ok = bench.timed(torch, None, wl, 10, 3)
    ms = float(np.mean(k))
    print(f"ok={ok} {ms:.3f} ms/step, {wl.out_bytes / ms / 1e6:.1f} GB/s decoded, "
          f"{(wl.in_bytes + wl.out_bytes) / ms / 1e6:.1f} GB/s traffic", flush=True)


if __name__ == "__main__":
    main()
