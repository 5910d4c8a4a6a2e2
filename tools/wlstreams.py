"""A multi-column bench workload (C3 or C5) timed under the stream mode of
bench.StreamSet that SB_BENCH_STREAMS selects (torch | own):
python tools/wlstreams.py c3|c5 [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    name = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    pa_amd.default_context(0)
    thr = bench.cpu_threads()
    if name == "c3":
        wl = bench.WorkloadC3(torch, pa_amd, 100_000_000, 77, 0, thr)
    else:
        wl = bench.WorkloadC5(torch, pa_amd, 8_388_608, 555, 0, thr)
    wall, k, ok = bench.timed(torch, None, wl, steps, 3)
    print(f"{name} streams={os.environ.get('SB_BENCH_STREAMS', 'default')}: ok={ok} wall {wall / steps * 1e3:.3f} ms/step, "
          f"event median {float(np.median(k)):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
