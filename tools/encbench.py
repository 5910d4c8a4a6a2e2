"""Device encode of C5-shaped LZ4 columns, timed per column kind:
python tools/encbench.py [rows] (PA_AMD_LIB selects a variant library)."""
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
    rng = np.random.default_rng(5)
    ctx = pa_amd.default_context(0)
    o = pa_amd.WriteOptions(default_compression=1, max_page_size=8192, seed=1)
    f = np.round(rng.standard_normal(rows) * 1e4, 2)
    svals, soffs = bench.decimal_strings(rng.integers(0, 10**6, rows))
    cases = {
        "f64_lz4": lambda: pa_amd.encode_column_device(tf, None, False, o, ctx=ctx),
        "utf8_lz4": lambda: pa_amd.encode_binary_column_device(ts, to, None, False, o, pa_amd.UTF8, ctx=ctx),
        "i32_rand_lz4": lambda: pa_amd.encode_column_device(ti, None, False, o, ctx=ctx),
    }
    tf = torch.from_numpy(f).cuda()
    ts = torch.from_numpy(np.frombuffer(svals, np.uint8).copy()).cuda()
    to = torch.from_numpy(soffs).cuda()
    ti = torch.from_numpy(rng.integers(0, 1 << 20, rows).astype(np.int32)).cuda()
    host = {"f64_lz4": lambda: pa_amd.encode_column(f, None, False, o),
            "utf8_lz4": lambda: pa_amd.encode_binary_column(svals, soffs, None, False, o, physical_type=pa_amd.UTF8),
            "i32_rand_lz4": lambda: pa_amd.encode_column(ti.cpu().numpy(), None, False, o)}
    for name, fn in cases.items():
        same = fn()[0].cpu().numpy().tobytes() == host[name]()[0]
        print(f"{name}: byte-identical to the host writer: {same}", flush=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            r = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        print(f"{name}: {dt * 1e3:.2f} ms, {len(r[0]) if not hasattr(r[0], 'numel') else r[0].numel()} bytes", flush=True)


if __name__ == "__main__":
    main()
