"""Kernel microbenchmark: decode-kernel time per workload shape, HIP events on
the launch stream, two rotating input/output copies.  Prints one row per
workload: kernel us, traffic GB/s (compressed in + decoded out), fraction of
8 TB/s.  Usage: python tools/kbench.py [rows] [workload ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

P = 8192


def gen(kind, rows, seed=1):
    rng = np.random.default_rng(seed)
    v = np.empty(rows, np.int32)
    for p in range((rows + P - 1) // P):
        n = min(P, rows - p * P)
        s = slice(p * P, p * P + n)
        if kind.startswith("b") and kind[1:].isdigit():
            v[s] = rng.integers(0, 1 << int(kind[1:]), n)
        elif kind == "bcycle":
            v[s] = rng.integers(0, 1 << (12 + (p * 7) % 13), n)
        elif kind == "rle":
            lens = rng.choice(np.array([2, 3]), size=n // 2 + 2, p=[0.3, 0.7])
            v[s] = np.repeat(rng.integers(0, 2**31, len(lens)), lens)[:n]
        elif kind == "rle_long":
            v[s] = np.repeat(rng.integers(0, 2**31, n // 64 + 2), 64)[:n]
        elif kind == "mix":
            if p % 5 == 4:
                lens = rng.choice(np.array([2, 3]), size=n // 2 + 2, p=[0.3, 0.7])
                v[s] = np.repeat(rng.integers(0, 2**31, len(lens)), lens)[:n]
            else:
                v[s] = rng.integers(0, 1 << (12 + (p * 7) % 13), n)
        elif kind == "dict":
            v[s] = rng.integers(0, 1000, n) * 7919
        elif kind == "delta":
            v[s] = np.cumsum(rng.integers(0, 64, n)).astype(np.int32)
        elif kind == "none":
            v[s] = rng.integers(-2**31, 2**31 - 1, n)
        else:
            raise ValueError(kind)
    return v


def main():
    import torch

    import pa_amd

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    kinds = sys.argv[2:] or ["b12", "b4", "b20", "b24", "bcycle", "rle", "rle_long", "mix", "dict", "delta", "none"]
    ctx = pa_amd.default_context(0)
    print(f"{'workload':10s} {'codecs':28s} {'MB in':>8s} {'kern us':>9s} {'GB/s':>8s} {'frac':>6s} {'dec GB/s':>9s} ok")
    for kind in kinds:
        v = gen(kind, rows)
        ratio = None if kind == "none" else 1.2
        chunk, metas = pa_amd.encode_column(v, None, False, pa_amd.WriteOptions(default_compress_ratio=ratio, max_page_size=P, seed=3))
        mix = {}
        pos = 0
        for m in metas:
            mix[chunk[pos]] = mix.get(chunk[pos], 0) + 1
            pos += m.length
        host = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy())
        decs = [pa_amd.ColumnDecoder(host.cuda(), metas, np.int32, False, ctx) for _ in range(2)]
        outs = [d.alloc_outputs() for d in decs]
        for k in range(4):
            decs[k & 1].decode_async(*outs[k & 1])
        torch.cuda.synchronize()
        for d in decs:
            d.check()
        ok = bool(torch.equal(outs[0][0][:rows].cpu(), torch.from_numpy(v)))
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for k, (a, b) in enumerate(evs):
            a.record()
            decs[k & 1].decode_async(*outs[k & 1])
            b.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
        traffic = (len(chunk) + rows * 4) / (ms / 1e3) / 1e9
        print(f"{kind:10s} {str(mix):28s} {len(chunk)/1e6:8.1f} {ms*1e3:9.1f} {traffic:8.1f} {traffic/8000:6.3f} {rows*4/(ms/1e3)/1e9:9.1f} {ok}", flush=True)
        del decs, outs, host


if __name__ == "__main__":
    main()
