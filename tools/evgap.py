"""Wall clock of a workload's steps with and without a HIP event after each
step (does the per-step marker cost device time between steps?):
python tools/evgap.py c2|c4 [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    name = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    pa_amd.default_context(0)
    thr = bench.cpu_threads()
    if name == "c2":
        wl = bench.Workload(torch, pa_amd, 100_000_000, 42, "mix", 0, thr)
    else:
        wl = bench.WorkloadC4(torch, pa_amd, 50_000_000, 99, 0, thr)
    for k in range(4):
        wl.step(k)
    torch.cuda.synchronize()
    for rep in range(3):
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evs[0].record()
        for k in range(steps):
            wl.step(k)
            evs[k + 1].record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for k in range(steps):
            wl.step(k)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(steps):
            wl.step(k)
        e1.record()
        torch.cuda.synchronize()
        ev = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(steps))
        print(f"{name} rep {rep}: per-step events wall {(t1 - t0) / steps * 1e3:.4f} ms (event median {ev[steps // 2]:.4f}); "
              f"no events wall {(t3 - t2) / steps * 1e3:.4f} ms; two events {e0.elapsed_time(e1) / steps:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
