"""C5 table encode on the device alone (bench.WorkloadC5's timed
encode_table_device, byte-checked against the host writer):
python tools/c5enc.py (PA_AMD_LIB selects a variant library)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    pa_amd.default_context(0)
    wl = bench.WorkloadC5(torch, pa_amd, 8_388_608, 555, 0, 16)
    print(f"c5 encode {wl.encode_gpu_s * 1e3:.1f} ms, {wl.raw_bytes / wl.encode_gpu_s / 1e9:.1f} GB/s, "
          f"byte-identical {wl.byte_identical}", flush=True)


if __name__ == "__main__":
    main()
