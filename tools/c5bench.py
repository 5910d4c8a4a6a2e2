"""Config-5 table alone (kernel trace target): python tools/c5bench.py [rows] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    wl = bench.WorkloadC5(torch, pa_amd, rows, 555, 0, 16)
    w, k, ok = bench.timed(torch, None, wl, steps, 2)
    print(f"c5: {w / steps * 1e3:.3f} ms/step, {wl.out_bytes * steps / w / 1e9:.1f} GB/s decoded, ok={ok}", flush=True)


if __name__ == "__main__":
    main()
