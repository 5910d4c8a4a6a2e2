"""bench.encode_gpu alone (C2 adaptive / forced Bitpacking / configs[0] None
device encodes, byte-checked against the host writer): python
tools/enc_c2.py [rows] (PA_AMD_LIB selects a variant library)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import pa_amd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    pa_amd.default_context(0)
    print(json.dumps(bench.encode_gpu(torch, pa_amd, rows, 0, 16, 20)), flush=True)


if __name__ == "__main__":
    main()
