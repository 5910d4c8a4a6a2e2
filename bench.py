#!/usr/bin/env python3
"""bench.py -- decoded GB/s of the MI355X strawboat page decoder.

Workload (BASELINE.json configs[1]): a non-nullable
Int32 column of 100M rows in 8192-row pages, written by the engine's writer
with the reference's adaptive codec choice at default_compress_ratio 1.2
(write/common.rs:49-119, compression/integer/mod.rs:231-308).  Page data
is shaped so the adaptive choice lands on the two codecs the config names:
80 % of pages uniform in [0, 2^b) with b cycling 12..24 (-> Bitpacking),
20 % runs of length 2-3 of random 31-bit values (-> RLE).  The codec of
every page is read back and reported.

A "step" = one batched decode of the whole column (compressed pages resident
in HBM -> Arrow values buffer in HBM).  value = decoded bytes of all ranks /
max-over-ranks wall time of the timed steps.  Weak scaling: each rank owns a
100M-row shard (its own page queue, no collectives on the data path).

Also reported: the all-Bitpacking b=12 variant (the north star's >=60 %
roofline target), the roofline of the decode kernel from HIP events on the
launch stream, and the CPU restatement (oracle, 1 thread) on the same column.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded GB/s (uncompressed) per node at 1/2/4/8 GPUs; bit-exact vs CPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PAGE_ROWS = 8192


def gen_c2(rows: int, seed: int, variant: str) -> np.ndarray:
    rng = np.random.default_rng(seed)
    v = np.empty(rows, np.int32)
    npg = (rows + PAGE_ROWS - 1) // PAGE_ROWS
    for p in range(npg):
        n = min(PAGE_ROWS, rows - p * PAGE_ROWS)
        s = slice(p * PAGE_ROWS, p * PAGE_ROWS + n)
        if variant == "b12":
            v[s] = rng.integers(0, 1 << 12, n)
        elif p % 5 == 4:
            lens = rng.choice(np.array([2, 3]), size=n // 2 + 2, p=[0.3, 0.7])
            v[s] = np.repeat(rng.integers(0, 2**31, len(lens)), lens)[:n]
        else:
            v[s] = rng.integers(0, 1 << (12 + (p * 7) % 13), n)
    return v


def codec_mix(chunk: bytes, metas) -> dict:
    names = {0: "none", 1: "lz4", 10: "rle", 11: "dict", 12: "one_value", 13: "freq", 14: "bitpacking",
             15: "delta_bitpacking"}
    mix, pos = {}, 0
    for m in metas:
        k = names.get(chunk[pos], str(chunk[pos]))
        mix[k] = mix.get(k, 0) + 1
        pos += m.length
    return mix


class Workload:
    """One encoded column resident in HBM twice (two input copies and two
    output buffers, alternated per step so the 256 MiB Infinity Cache cannot
    serve a step from the previous one)."""

    def __init__(self, torch, pa, rows, seed, variant, device, threads):
        t0 = time.time()
        self.values = gen_c2(rows, seed, variant)
        opts = pa.WriteOptions(default_compress_ratio=1.2, max_page_size=PAGE_ROWS, seed=seed)
        self.chunk, self.metas = pa.encode_column(self.values, None, False, opts, n_threads=threads)
        self.encode_s = time.time() - t0
        self.mix = codec_mix(self.chunk, self.metas)
        self.rows = rows
        self.in_bytes = len(self.chunk)
        self.out_bytes = rows * 4
        dev = f"cuda:{device}"
        host = torch.from_numpy(np.frombuffer(self.chunk, dtype=np.uint8).copy())
        self.decs, self.outs = [], []
        for _ in range(2):
            d = pa.ColumnDecoder(host.to(dev), self.metas, np.int32, False)
            self.decs.append(d)
            self.outs.append(d.alloc_outputs())
        self.expect = torch.from_numpy(self.values).to(dev)
        torch.cuda.synchronize()

    def step(self, k):
        d = self.decs[k & 1]
        d.decode_async(*self.outs[k & 1])

    def verify(self, torch) -> bool:
        ok = True
        for d, (v, _) in zip(self.decs, self.outs):
            d.check()
            ok &= bool(torch.equal(v[: self.rows], self.expect))
        return ok


def timed(torch, dist, wl: Workload, steps: int, warmup: int):
    for k in range(warmup):
        wl.step(k)
    torch.cuda.synchronize()
    ok = wl.verify(torch)
    # HIP events on the launch stream (the context launches on torch's current
    # stream) bracket the whole timed region: per-launch average = span / steps
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for k in range(steps):
        wl.step(k)
    ev1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    for d in wl.decs:
        d.check()
    kern_ms = [ev0.elapsed_time(ev1) / steps]
    return t1 - t0, kern_ms, ok


def cpu_baseline(wl: Workload, budget_s: float = 10.0) -> dict:
    from oracle import oracle as O

    metas = [(m.length, m.num_values) for m in wl.metas]
    t0 = time.perf_counter()
    out, _ = O.read_column(wl.chunk, metas, np.int32)
    first = time.perf_counter() - t0
    assert np.array_equal(out, wl.values), "oracle decode mismatch"
    passes = max(1, min(50, int(math.ceil(budget_s / max(first, 1e-3))) - 1))
    t0 = time.perf_counter()
    for _ in range(passes):
        O.read_column(wl.chunk, metas, np.int32)
    dt = time.perf_counter() - t0
    return {
        "value": round(wl.out_bytes * passes / dt / 1e9, 3),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle/ C restatement of read_integer over the full {wl.rows}-row column, {passes} passes "
                  f"({dt:.1f} s), 1 thread, compressed pages in host RAM -> values in host RAM",
    }


def decimal_strings(vals: np.ndarray):
    """Decimal strings of non-negative ints (tests/it/io.rs:385-397 shape),
    vectorized: -> (values bytes, int64 offsets)."""
    v = vals.astype(np.int64)
    nd = np.ones(len(v), np.int64)
    for k in range(1, 19):
        nd += v >= 10**k
    offs = np.zeros(len(v) + 1, np.int64)
    np.cumsum(nd, out=offs[1:])
    out = np.empty(int(offs[-1]), np.uint8)
    pos = offs[1:] - 1  # last digit of each row
    x = v.copy()
    left = nd.copy()
    while True:
        m = left > 0
        if not m.any():
            break
        out[pos[m]] = (48 + x[m] % 10).astype(np.uint8)
        x[m] //= 10
        pos[m] -= 1
        left[m] -= 1
    return out.tobytes(), offs


class WorkloadC3:
    """BASELINE.json configs[2]: nullable Float64 + nullable Utf8, LZ4 pages,
    ratio None (always the general codec), 10 % nulls, 8192-row pages.
    A step decodes both columns; two input/output copies rotate."""

    def __init__(self, torch, pa, rows, seed, device, threads):
        rng = np.random.default_rng(seed)
        self.rows = rows
        f = np.round(rng.standard_normal(rows) * 1e4, 2)
        fvalid = rng.random(rows) >= 0.1
        svals, soffs = decimal_strings(rng.integers(0, 10**6, rows))
        svalid = rng.random(rows) >= 0.1
        opts = pa.WriteOptions(default_compression=1, default_compress_ratio=None, max_page_size=PAGE_ROWS, seed=seed)
        self.fchunk, self.fmetas = pa.encode_column(f, fvalid, True, opts, n_threads=threads)
        self.schunk, self.smetas = pa.encode_binary_column(svals, soffs, svalid, True, opts, physical_type=pa.UTF8,
                                                           n_threads=threads)
        dev = f"cuda:{device}"
        fh = torch.from_numpy(np.frombuffer(self.fchunk, np.uint8).copy())
        sh = torch.from_numpy(np.frombuffer(self.schunk, np.uint8).copy())
        self.fdec = [pa.ColumnDecoder(fh.to(dev), self.fmetas, np.float64, True) for _ in range(2)]
        self.sdec = [pa.BinaryColumnDecoder(sh.to(dev), self.smetas, pa.UTF8, True) for _ in range(2)]
        self.fout = [d.alloc_outputs() for d in self.fdec]
        self.sout = [d.alloc_outputs() for d in self.sdec]
        self.in_bytes = len(self.fchunk) + len(self.schunk)
        nb = (rows + 7) // 8
        self.out_bytes = rows * 8 + nb + 4 * (rows + 1) + len(svals) + nb
        self.exp = (torch.from_numpy(f.view(np.int64)).to(dev), torch.from_numpy(np.packbits(fvalid, bitorder="little")).to(dev),
                    torch.from_numpy(soffs.astype(np.int32)).to(dev), torch.from_numpy(np.frombuffer(svals, np.uint8).copy()).to(dev),
                    torch.from_numpy(np.packbits(svalid, bitorder="little")).to(dev))
        torch.cuda.synchronize()

    def step(self, k):
        self.fdec[k & 1].decode_async(*self.fout[k & 1])
        self.sdec[k & 1].decode_async(*self.sout[k & 1])

    def verify(self, torch) -> bool:
        ok = True
        nb = (self.rows + 7) // 8
        for i in range(2):
            self.fdec[i].check()
            self.sdec[i].check()
            fv, fm = self.fout[i]
            so, sv, sm = self.sout[i]
            ok &= bool(torch.equal(fv[: self.rows], self.exp[0]))
            ok &= bool(torch.equal(fm[:nb], self.exp[1]))
            ok &= bool(torch.equal(so, self.exp[2]))
            ok &= bool(torch.equal(sv[: self.exp[3].numel()], self.exp[3]))
            ok &= bool(torch.equal(sm[:nb], self.exp[4]))
        return ok

    @property
    def decs(self):
        return self.fdec + self.sdec


class WorkloadC4:
    """BASELINE.json configs[3]: List<Int32>, nullable lists (10 %) of
    nullable items (20 %), lengths uniform in {0, 1, 2} (tests/it/io.rs:399-415
    shape), items uniform in [0, 2^16), adaptive ratio 1.2, 8192-row pages.
    A step = sizing pass + level decode (offsets, both bitmaps) + values."""

    def __init__(self, torch, pa, rows, seed, device, threads):
        rng = np.random.default_rng(seed)
        self.rows = rows
        lens = rng.integers(0, 3, rows)
        lv = rng.random(rows) >= 0.1
        lens[~lv] = 0
        offs = np.zeros(rows + 1, np.int64)
        np.cumsum(lens, out=offs[1:])
        V = int(offs[-1])
        child = rng.integers(0, 1 << 16, V).astype(np.int32)
        cv = rng.random(V) >= 0.2
        opts = pa.WriteOptions(default_compress_ratio=1.2, max_page_size=PAGE_ROWS, seed=seed)
        self.chunk, self.metas = pa.encode_list_column(offs, child, lv, cv, True, True, opts, n_threads=threads)
        self.mix = {}
        dev = f"cuda:{device}"
        h = torch.from_numpy(np.frombuffer(self.chunk, np.uint8).copy())
        self.decs = [pa.ListColumnDecoder(h.to(dev), self.metas, np.int32, True, True) for _ in range(2)]
        self.outs = [d.alloc_outputs() for d in self.decs]
        self.leaves = V
        self.in_bytes = len(self.chunk)
        self.out_bytes = 4 * (rows + 1) + (rows + 7) // 8 + 4 * V + (V + 7) // 8
        self.exp = (torch.from_numpy(offs.astype(np.int32)).to(dev), torch.from_numpy(np.packbits(lv, bitorder="little")).to(dev),
                    torch.from_numpy(child).to(dev), torch.from_numpy(np.packbits(cv, bitorder="little")).to(dev),
                    torch.from_numpy(cv).to(dev))
        torch.cuda.synchronize()

    def step(self, k):
        self.decs[k & 1].decode_async(*self.outs[k & 1])

    def verify(self, torch) -> bool:
        ok = True
        for d, (o, lv, v, fv) in zip(self.decs, self.outs):
            d.check()
            ok &= bool(torch.equal(o, self.exp[0]))
            ok &= bool(torch.equal(lv[: self.exp[1].numel()], self.exp[1]))
            ok &= bool(torch.equal(fv[: self.exp[3].numel()], self.exp[3]))
            m = self.exp[4]
            ok &= bool(torch.equal(v[: self.leaves][m], self.exp[2][m]))
        return ok


def load_traffic(workload: str):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get(workload)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-b12", action="store_true", help="skip the all-bitpack b=12 variant")
    ap.add_argument("--no-c3", action="store_true", help="skip the config-3 (Float64 + Utf8, LZ4) workload")
    ap.add_argument("--c3-rows", type=int, default=100_000_000)
    ap.add_argument("--no-c4", action="store_true", help="skip the config-4 (List<Int32>) workload")
    ap.add_argument("--c4-rows", type=int, default=50_000_000)
    args = ap.parse_args()

    import torch

    import pa_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as tdist

        tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        dist = tdist
    threads = max(1, min(16, (os.cpu_count() or 8) // max(world, 1)))
    pa_amd.default_context(local)

    wl = Workload(torch, pa_amd, args.rows, 42 + rank, "mix", local, threads)
    wall, kern_ms, ok = timed(torch, dist, wl, args.steps, args.warmup)
    t = torch.tensor([wall, 0.0 if ok else 1.0], device=f"cuda:{local}", dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max, any_bad = float(t[0]), bool(t[1] > 0)
    kavg = float(np.mean(kern_ms))
    achieved = (wl.in_bytes + wl.out_bytes) / (kavg / 1e3) / 1e9
    value = world * wl.out_bytes * args.steps / wall_max / 1e9

    extra = {}
    if not args.no_b12:
        wl12 = Workload(torch, pa_amd, args.rows, 4242 + rank, "b12", local, threads)
        w12, k12, ok12 = timed(torch, dist, wl12, args.steps, args.warmup)
        k12avg = float(np.mean(k12))
        a12 = (wl12.in_bytes + wl12.out_bytes) / (k12avg / 1e3) / 1e9
        extra["bitpack_b12"] = {
            "decoded_GBps": round(wl12.out_bytes * args.steps / w12 / 1e9, 1),
            "kernel_ms": round(k12avg, 4),
            "kernel_traffic_GBps": round(a12, 1),
            "roofline_frac": round(a12 / HBM_PEAK_GBPS, 4),
            "compressed_bytes": wl12.in_bytes,
            "bit_exact": bool(ok12),
        }
        del wl12

    if not args.no_c3:
        wl3 = WorkloadC3(torch, pa_amd, args.c3_rows, 77 + rank, local, threads)
        w3, k3, ok3 = timed(torch, dist, wl3, max(3, args.steps // 4), args.warmup)
        steps3 = max(3, args.steps // 4)
        extra["c3_f64_utf8_lz4_nullable"] = {
            "rows": args.c3_rows,
            "decoded_GBps": round(wl3.out_bytes * steps3 / w3 / 1e9, 1),
            "ms_per_step": round(w3 / steps3 * 1e3, 3),
            "step_traffic_GBps": round((wl3.in_bytes + wl3.out_bytes) / (float(np.mean(k3)) / 1e3) / 1e9, 1),
            "roofline_frac": round((wl3.in_bytes + wl3.out_bytes) / (float(np.mean(k3)) / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
            "compressed_bytes": wl3.in_bytes,
            "decoded_bytes": wl3.out_bytes,
            "bit_exact": bool(ok3),
            "kernels": "k_decode_staged<8,true> + k_decode_deferred<8,true> (LZ4) + k_bin_decode<4>",
        }
        del wl3

    if not args.no_c4:
        wl4 = WorkloadC4(torch, pa_amd, args.c4_rows, 99 + rank, local, threads)
        steps4 = max(3, args.steps // 2)
        w4, k4, ok4 = timed(torch, dist, wl4, steps4, args.warmup)
        t4 = torch.tensor([w4], device=f"cuda:{local}", dtype=torch.float64)
        if dist:
            dist.all_reduce(t4, op=dist.ReduceOp.MAX)
        k4avg = float(np.mean(k4))
        a4 = (wl4.in_bytes + wl4.out_bytes) / (k4avg / 1e3) / 1e9
        extra["c4_list_int32_nested"] = {
            "rows_per_gpu": args.c4_rows,
            "leaves_per_gpu": wl4.leaves,
            "pages_per_gpu": len(wl4.metas),
            "decoded_GBps": round(world * wl4.out_bytes * steps4 / float(t4[0]) / 1e9, 1),
            "ms_per_step": round(float(t4[0]) / steps4 * 1e3, 3),
            "step_traffic_GBps": round(a4, 1),
            "roofline_frac": round(a4 / HBM_PEAK_GBPS, 4),
            "compressed_bytes_per_gpu": wl4.in_bytes,
            "decoded_bytes_per_gpu": wl4.out_bytes,
            "bit_exact": bool(ok4),
            "parallelism": f"page-shard x{world}",
            "kernels": "k_list_size + k_list_scan + k_list_levels + k_decode_staged<4,false>",
        }
        del wl4

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded numpy; pages encoded by the engine's writer)",
            "config": {
                "workload": "c2_int32_adaptive_bitpack_rle",
                "rows_per_gpu": args.rows,
                "page_rows": PAGE_ROWS,
                "pages_per_gpu": len(wl.metas),
                "codec_mix": wl.mix,
                "compress_ratio_option": 1.2,
                "compressed_bytes_per_gpu": wl.in_bytes,
                "decoded_bytes_per_gpu": wl.out_bytes,
                "parallelism": f"page-shard x{world}",
            },
            "bit_exact": (not any_bad),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic("c2_int32_adaptive_bitpack_rle"),
                "kernel": "k_decode_staged<4,false>",
                "kernel_ms": round(kavg, 4),
                "bytes_per_launch": wl.in_bytes + wl.out_bytes,
            },
        }
        line.update(extra)
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(wl)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
