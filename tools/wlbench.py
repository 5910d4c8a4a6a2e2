"""One bench workload alone (for per-workload rocprof kernel splits):
python tools/wlbench.py c3|c4|c5 [steps] [warmup].  Builds bench.py's
WorkloadC3 / C4 / C5 at the bench's default size and seed, times `steps`
steps after `warmup`, prints ms/step and the step's kernel launches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    wl_name = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    pa_amd.default_context(0)
    thr = bench.cpu_threads()
    if wl_name == "c3":
        wl = bench.WorkloadC3(torch, pa_amd, 100_000_000, 77, 0, thr)
    elif wl_name == "c4":
        wl = bench.WorkloadC4(torch, pa_amd, 50_000_000, 99, 0, thr)
    else:
        wl = bench.WorkloadC5(torch, pa_amd, 8_388_608, 555, 0, thr)
    print(f"{wl_name}: built", flush=True)
    wall, k, ok = bench.timed(torch, None, wl, steps, warm)
    ms = float(np.mean(k))
    print(f"{wl_name}: ok={ok} {ms:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
