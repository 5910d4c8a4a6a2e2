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


# ---- tests/golden/columns.npz: the non-fixed-width families ----------------
# Binary / Utf8 (Basic under each general codec, Dict, Freq, OneValue, the
# adaptive choice), Boolean (Basic, RLE, OneValue), List<Int32>, List<Utf8>,
# a Struct and a Map field -- multi-page column chunks written page by page by
# the oracle's writer, page p sampled with sb_page_seed(7, p) as the product
# writer does, and their decoded Arrow buffers as the oracle reads them.
import json  # noqa: E402

from oracle import nest as NE  # noqa: E402

M64 = (1 << 64) - 1


def page_seed(seed, page):
    """sb_page_seed (pa_amd/csrc/sb_encode.cpp page_seed): one splitmix64 step."""
    s = (seed ^ ((page * 0xD1B54A32D192ED03) & M64)) & M64
    z = (s + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


SEED = 7
COLS = {}


def opts_for(name, dc, p):
    kw = {"plain": dict(), "adaptive": dict(ratio=2.0), "rle": dict(ratio=1.0, forced=O.RLE),
          "dict": dict(ratio=1.0, forced=O.DICT), "freq": dict(ratio=1.0, forced=O.FREQ),
          "onevalue": dict(ratio=2.0)}[name]
    return O.WriteOptions.make(default_codec=dc, seed=page_seed(SEED, p), **kw)


def put(case, **arrays):
    for k, v in arrays.items():
        if v is not None:
            COLS[f"{case}__{k}"] = np.asarray(v)


crng = np.random.default_rng(77)
N_ROWS, STEP = 1500, 500
GENERAL = [("plain", 0, ""), ("plain", 1, "_lz4"), ("plain", 2, "_zstd"), ("plain", 3, "_snappy")]
for large in (False, True):
    for nullable in (False, True):
        for name, dc, cname in GENERAL + [("dict", 0, ""), ("freq", 0, ""), ("onevalue", 0, ""), ("adaptive", 0, ""),
                                          ("adaptive", 1, "_lz4")]:
            if name in ("dict", "adaptive"):
                ints = crng.integers(0, 40, N_ROWS)
            elif name == "freq":
                ints = np.where(crng.random(N_ROWS) < 0.95, 777, crng.integers(0, 10 ** 6, N_ROWS))
            elif name == "onevalue":
                ints = np.full(N_ROWS, 4242)
            else:
                ints = crng.integers(0, 10 ** 6, N_ROWS)
            strs = [("é%d" % x if x % 7 == 0 else "%d" % x).encode() for x in ints]
            valid = crng.random(N_ROWS) > 0.2 if nullable else None
            if valid is not None:
                strs = [s if v else b"" for s, v in zip(strs, valid)]
            vals, offs = O.strings_to_arrow(strs)
            pages, metas = [], []
            for p, r0 in enumerate(range(0, N_ROWS, STEP)):
                r1 = min(N_ROWS, r0 + STEP)
                pg = O.write_binary_page(vals, offs[r0:r1 + 1], None if valid is None else valid[r0:r1], nullable,
                                         opts_for(name, dc, p), 8 if large else 4, len(vals))
                pages.append(pg)
                metas.append((len(pg), r1 - r0))
            chunk = b"".join(pages)
            eo, ev, evalid = O.read_binary_column(chunk, metas, nullable, 8 if large else 4)
            case = f"bin_{'largebin' if large else 'utf8'}_{'null' if nullable else 'req'}_{name}{cname}"
            put(case, chunk=np.frombuffer(chunk, np.uint8), metas=np.asarray(metas, np.uint64),
                in_values=np.frombuffer(vals, np.uint8), in_offsets=offs, in_validity=valid,
                offsets=eo, values=np.frombuffer(ev, np.uint8), validity=evalid)

for nullable in (False, True):
    for name, dc, cname, step in [(n_, d_, c_, 504) for n_, d_, c_ in GENERAL] + [
            ("plain", 0, "_ragged", 500), ("plain", 1, "_lz4_ragged", 500), ("rle", 0, "", 504),
            ("onevalue", 0, "", 504), ("adaptive", 0, "", 504)]:
        if name == "onevalue":
            bits = np.ones(N_ROWS, bool)
        elif name in ("rle", "adaptive"):
            bits = np.repeat(crng.random(N_ROWS // 50 + 1) < 0.5, 50)[:N_ROWS]
        else:
            bits = crng.random(N_ROWS) < 0.5
        valid = crng.random(N_ROWS) > 0.2 if nullable else None
        pages, metas = [], []
        for p, r0 in enumerate(range(0, N_ROWS, step)):
            r1 = min(N_ROWS, r0 + step)
            pg = O.write_bool_page(bits, None if valid is None else valid[r0:r1], nullable, opts_for(name, dc, p),
                                   offset=r0, n=r1 - r0)
            pages.append(pg)
            metas.append((len(pg), r1 - r0))
        chunk = b"".join(pages)
        ev, evalid = O.read_bool_column(chunk, metas, nullable)
        case = f"bool_{'null' if nullable else 'req'}_{name}{cname}"
        put(case, chunk=np.frombuffer(chunk, np.uint8), metas=np.asarray(metas, np.uint64), in_values=bits,
            in_validity=valid, step=np.asarray(step), values=ev, validity=evalid)


def f_json(f):
    return {"kind": f.kind, "nullable": f.nullable, "leaf": f.leaf, "dtype": None if f.dtype is None else f.dtype.str,
            "large": f.large, "name": f.name, "children": [f_json(c) for c in f.children]}


def gen_leaf(f, n, rng, live=None):
    pv = np.ones(n, bool) if live is None else live
    valid = (rng.random(n) > 0.2) & pv if f.nullable else None
    alive = pv if valid is None else valid
    if f.kind == "leaf":
        if f.leaf == "binary":
            strs = [b"%d" % x if a else b"" for x, a in zip(rng.integers(0, 60, n), alive)]
            v, o = O.strings_to_arrow(strs)
            return NE.A("leaf", n, valid, values=(o, v))
        if f.leaf == "bool":
            return NE.A("leaf", n, valid, values=(rng.random(n) < 0.5) & alive)
        return NE.A("leaf", n, valid, values=np.where(alive, rng.integers(0, 5000, n), 0).astype(f.dtype))
    if f.kind == "struct":
        return NE.A("struct", n, valid, children=[gen_leaf(c, n, rng, alive) for c in f.children])
    lens = np.where(alive, rng.integers(0, 4, n), 0)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    return NE.A(f.kind, n, valid, offsets=offs, children=[gen_leaf(f.children[0], int(offs[-1]), rng)])


i32 = lambda nul, name="": NE.F("leaf", nul, leaf="fixed", dtype=np.dtype(np.int32), name=name)  # noqa: E731
utf8 = lambda nul, name="": NE.F("leaf", nul, leaf="binary", name=name)  # noqa: E731
NESTED = {
    "list_i32": NE.F("list", True, [i32(True, "item")]),
    "list_utf8": NE.F("list", True, [utf8(True, "item")]),
    "struct": NE.F("struct", True, [NE.F("leaf", True, leaf="binary", large=True, name="name"), i32(True, "age"),
                                    NE.F("leaf", True, leaf="bool", name="flag")]),
    "map": NE.F("map", True, [NE.F("struct", False, [i32(False, "key"), utf8(True, "value")], name="entries")]),
}
for fname, f in NESTED.items():
    for name, dc, cname in [("plain", 0, ""), ("plain", 1, "_lz4"), ("plain", 2, "_zstd"), ("adaptive", 0, "")]:
        a = gen_leaf(f, N_ROWS, crng)
        cols = NE.write_field(f, a, STEP, opts_for(name, dc, 0), page_seed=lambda p: page_seed(SEED, p))
        case = f"nest_{fname}_{name}{cname}"
        put(case, field=np.asarray(json.dumps(f_json(f))))
        for k, (path, (chunk, metas)) in enumerate(zip(NE.leaf_paths(f), cols)):
            r = NE.read_leaf(path, chunk, metas)
            lv = r["values"]
            arrs = dict(chunk=np.frombuffer(chunk, np.uint8), metas=np.asarray(metas, np.uint64),
                        leaf_validity=r["leaf_validity"], counts=np.asarray(r["counts"], np.uint64))
            if isinstance(lv, tuple):
                arrs.update(values_offsets=lv[0], values=np.frombuffer(lv[1], np.uint8))
            else:
                arrs.update(values=lv)
            for d, (o, v) in enumerate(zip(r["offsets"], r["validity"])):
                arrs[f"offsets{d}"] = o
                arrs[f"validity{d}"] = v
            put(f"{case}__{k}", **arrs)
        # the written array, node by node in pre-order, for the product writer's check
        nodes = []

        def walk(x):
            nodes.append(x)
            for c in x.children:
                walk(c)
        walk(a)
        for i, x in enumerate(nodes):
            src = dict(validity=x.validity, offsets=x.offsets, length=np.asarray(x.length))
            if x.kind == "leaf":
                if isinstance(x.values, tuple):
                    src.update(values_offsets=x.values[0], values=np.frombuffer(x.values[1], np.uint8))
                else:
                    src.update(values=x.values)
            put(f"{case}__node{i}", **src)

np.savez_compressed(os.path.join(ROOT, "tests", "golden", "columns.npz"), **COLS)
print(len({k.split("__")[0] for k in COLS}), "column cases")
