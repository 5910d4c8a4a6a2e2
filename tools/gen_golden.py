"""Generates tests/golden/pages.npz: small strawboat pages, one per
(type, codec, nullability) case, with their decoded values and validity.

The reference publishes no golden vectors; these pages
are written by the oracle's restatement of the reference writer with forced
codecs and a fixed sampler seed, and pinned so any later change to the
oracle, the product encoder or the GPU decoder shows up as a diff.
Run: python tools/gen_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

CASES = []
rng = np.random.default_rng(2024)
for dtype in ["int32", "uint32", "int64", "int8", "uint16", "float64", "float32"]:
    dt = np.dtype(dtype)
    n = 1024
    if dt.kind == "f":
        base = np.round(rng.standard_normal(n) * 100, 2).astype(dt)
        lowcard = rng.integers(0, 8, n).astype(dt)
    else:
        hi = min(2**31, np.iinfo(dt).max)
        base = rng.integers(0, min(hi, 5000), n).astype(dt)
        lowcard = rng.integers(0, 8, n).astype(dt)
    for nullable in (False, True):
        valid = rng.random(n) > 0.25 if nullable else None
        forced = [("plain", dict(ratio=None)), ("adaptive", dict(ratio=1.2)),
                  ("rle", dict(ratio=1.0, forced=O.RLE)), ("dict", dict(ratio=1.0, forced=O.DICT)),
                  ("freq", dict(ratio=1.0, forced=O.FREQ))]
        if dt.kind in "iu" and dt.itemsize == 4:
            forced.append(("bitpacking", dict(ratio=0.001, forced=O.BITPACKING)))
        if dt == np.float64:
            forced.append(("patas", dict(ratio=1.0, forced=O.PATAS)))
        for dc, cname in [(0, ""), (1, "_lz4"), (2, "_zstd"), (3, "_snappy")]:
            if dc:
                opts_list = [("plain", dict(ratio=None))]
            else:
                opts_list = forced
            for name, kw in opts_list:
                data = lowcard if name in ("dict", "freq", "rle") else base
                if name == "freq":
                    data = np.where(rng.random(n) < 0.95, data.dtype.type(3 if dt.kind == "f" or dt.itemsize == 1 else 300), data)
                opts = O.WriteOptions.make(default_codec=dc, seed=7, **kw)
                page = O.write_page(data, valid, nullable, opts)
                vals, vv = O.read_page(page, n, dt, nullable)
                CASES.append((f"{dtype}_{'null' if nullable else 'req'}_{name}{cname}", dtype, nullable, page, vals, vv, data))

out = {}
for key, dtype, nullable, page, vals, vv, data in CASES:
    out[key + "__page"] = np.frombuffer(page, np.uint8)
    out[key + "__values"] = vals
    out[key + "__input"] = data
    if nullable:
        out[key + "__validity"] = vv
os.makedirs(os.path.join(ROOT, "tests", "golden"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "pages.npz"), **out)
print(len(CASES), "cases")
