"""One bench workload alone (for per-workload rocprof kernel splits and PMC
passes): python tools/wlbench.py c2|c2h|c3|c4|c5 [steps] [warmup] [bytes.json].
Builds bench.py's Workload / WorkloadC3 / C4 / C5 at the bench's default
size and seed, times `steps` steps after `warmup`, prints ms/step, and
(optionally: a PMC window of `steps` more steps between two marker
launches) writes the workload's algorithmic bytes per step -- compressed
bytes read and Arrow bytes written, per column -- for the PMC summaries."""
import json
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
    cols = {}
    if wl_name == "c2":
        wl = bench.Workload(torch, pa_amd, 100_000_000, 42, "mix", 0, thr)
        cols["int32"] = (wl.in_bytes, wl.out_bytes)
    elif wl_name == "c2h":
        wl = bench.Workload(torch, pa_amd, 100_000_000, 4343, "hard", 0, thr)
        cols["int32"] = (wl.in_bytes, wl.out_bytes)
    elif wl_name == "c3":
        wl = bench.WorkloadC3(torch, pa_amd, 100_000_000, 77, 0, thr)
        nb = (wl.rows + 7) // 8
        cols["float64"] = (len(wl.fchunk), wl.rows * 8 + nb)
        cols["utf8"] = (len(wl.schunk), 4 * (wl.srows + 1) + wl.svals_len + (wl.srows + 7) // 8)
    elif wl_name == "c4":
        wl = bench.WorkloadC4(torch, pa_amd, 50_000_000, 99, 0, thr)
        cols["list_int32"] = (wl.in_bytes, wl.out_bytes)
    else:
        wl = bench.WorkloadC5(torch, pa_amd, 8_388_608, 555, 0, thr)
        cols["table"] = (wl.in_bytes, wl.out_bytes)
    print(f"{wl_name}: built", flush=True)
    wall, k, ok = bench.timed(torch, None, wl, steps, warm)
    ms = float(np.mean(k))
    print(f"{wl_name}: ok={ok} {ms:.3f} ms/step", flush=True)
    if len(sys.argv) > 4:
        # the PMC window: `steps` more steps between two marker launches (an
        # int16 arange), so tools/pmc_summary.py attributes exactly those
        # dispatches -- of every kernel, however many per step -- to the steps
        torch.cuda.synchronize()
        torch.arange(5, dtype=torch.int16, device="cuda")
        for s in range(steps):
            wl.step(s)
        torch.arange(5, dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
    if len(sys.argv) > 4:
        json.dump({"workload": wl_name, "ms_per_step": ms, "steps": steps, "in_bytes": wl.in_bytes, "out_bytes": wl.out_bytes,
                   "columns": {c: {"in_bytes": i, "out_bytes": o} for c, (i, o) in cols.items()}},
                  open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
