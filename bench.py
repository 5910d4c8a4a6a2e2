#!/usr/bin/env python3
"""bench.py -- decoded GB/s of the MI355X strawboat page decoder.

Workload (BASELINE.json configs[1]): a non-nullable
Int32 column of 100M rows in 8192-row pages, written by the engine's writer
with the reference's adaptive codec choice at default_compress_ratio 1.2
(write/common.rs:49-119, compression/integer/mod.rs:231-308).  Page data is
shaped as SURVEY.md §8(d) specifies: 80 % of pages uniform in [0, 2^b) with
b cycling 1..24, 20 % runs of 64-512 copies of random values.  The adaptive
choice then lands on Bitpacking for the uniform pages and on Dict -- not
RLE -- for the run pages and some low-width pages: with at most 128 distinct
values Dict's size estimate drops the index bytes to zero (dict.rs:109-120,
integer division) and its ratio beats RLE's sampled one.  The codec of every
page is read back and reported (workload "c2_int32_adaptive_bitpack_dict");
RLE throughput is measured by the c2_hard_mix variant (RLE runs of 2-3).

A "step" = one batched decode of the whole column (compressed pages resident
in HBM -> Arrow values buffer in HBM).  value = decoded bytes of all ranks /
max-over-ranks wall time of the timed steps.  Weak scaling: each rank owns a
100M-row shard (its own page queue, no collectives on the data path).

Also reported: the all-Bitpacking b=12 variant (the north star's >=60 %
roofline target), the harder C2 mix, configs 3-5 (Float64 + Utf8 under LZ4;
List<Int32>; the 64-column mixed table, encoded on the GPU and checked byte
for byte against the host writer), device encode rates, and per config the
CPU restatement of the reference's src/read decoder (oracle/, the
reference's algorithms with system liblz4 / libzstd) timed on 1 host thread
(the reference's shape) and on all the box's cores (pages sharded over
threads), with the CPU model.
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


BLOCK_PAGES = 64  # pages per generator / writer call (any rank can rebuild any block)


def page_rng(seed: int, p: int):
    """Page p's own generator: a column's pages are reproducible one by one."""
    return np.random.default_rng([seed, p])


def c2_page(variant: str, seed: int, p: int, n: int) -> np.ndarray:
    """Page p of SURVEY.md §8(d) C2: variant "mix" (b cycling 1..24 on 4 of
    5 pages, RLE runs of 64-512 on the fifth); "hard": b cycling 12..24 and
    RLE runs of 2-3 (more input bytes and 8x the runs); "b12": 12-bit."""
    rng = page_rng(seed, p)
    if variant == "b12":
        return rng.integers(0, 1 << 12, n).astype(np.int32)
    if p % 5 == 4:
        if variant == "hard":
            lens = rng.choice(np.array([2, 3]), size=n // 2 + 2, p=[0.3, 0.7])
        else:
            lens = rng.integers(64, 513, n // 64 + 2)
        return np.repeat(rng.integers(0, 2**31, len(lens)), lens)[:n].astype(np.int32)
    b = 12 + (p * 7) % 13 if variant == "hard" else 1 + (p - p // 5) % 24
    return rng.integers(0, 1 << b, n).astype(np.int32)


def gen_c2(rows: int, seed: int, variant: str, row0: int = 0) -> np.ndarray:
    """Rows [row0, row0 + rows) of the C2 column (row0 on a page boundary)."""
    p0 = row0 // PAGE_ROWS
    npg = (rows + PAGE_ROWS - 1) // PAGE_ROWS
    return np.concatenate([c2_page(variant, seed, p0 + i, min(PAGE_ROWS, rows - i * PAGE_ROWS)) for i in range(npg)]) \
        if rows else np.zeros(0, np.int32)


class ShardedColumn:
    """This rank's page shard of ONE column of `total_rows` rows (SURVEY.md
    §8(e)): the column is cut into blocks of BLOCK_PAGES pages, block b built
    by make_block(b, row0, rows) -> (payload, chunk bytes, [PageMeta]) from
    its own seeds, so any rank can rebuild any block.  Every rank builds a
    provisional row-balanced range of blocks, the ranks all-gather their page
    metas (setup only), pa_amd.shard_pages cuts the whole column into
    contiguous byte-balanced page ranges, and this rank keeps its range
    (building the blocks its range borrows).  `chunk` / `metas` are the
    shard's bytes and pages, `shard` the pa_amd.Shard the decoders take
    (for_shard), `pages` the (block, page-in-block) of each local page."""

    def __init__(self, pa, dist, world, rank, total_rows, make_block):
        br = BLOCK_PAGES * PAGE_ROWS
        nb = max(1, (total_rows + br - 1) // br)
        self.blocks = {}

        def get(b):
            if b not in self.blocks:
                r0 = b * br
                self.blocks[b] = make_block(b, r0, min(br, total_rows - r0))
            return self.blocks[b]

        prov = range(rank * nb // world, (rank + 1) * nb // world)
        known = {b: [(m.length, m.num_values) for m in get(b)[2]] for b in prov}
        if dist is not None and world > 1:
            parts = [None] * world
            dist.all_gather_object(parts, known)
            for d in parts:
                known.update(d)
        metas = [pa.PageMeta(ln, nv) for b in range(nb) for ln, nv in known[b]]
        sh = pa.shard_pages(metas, world)[rank]
        chunks, self.metas, self.pages = [], [], []
        if sh.page_end > sh.page_begin:
            for b in range(sh.page_begin // BLOCK_PAGES, (sh.page_end - 1) // BLOCK_PAGES + 1):
                _, chunk, bm = get(b)
                off = 0
                for j, m in enumerate(bm):
                    if sh.page_begin <= b * BLOCK_PAGES + j < sh.page_end:
                        chunks.append(chunk[off:off + m.length])
                        self.metas.append(m)
                        self.pages.append((b, j))
                    off += m.length
        for b in [b for b in self.blocks if not any(b == x for x, _ in self.pages)]:
            del self.blocks[b]
        self.chunk = b"".join(chunks)
        self.global_shard = sh
        self.shard = pa.Shard(rank, 0, len(self.metas), 0, len(self.chunk), sh.row_offset, sh.rows)
        self.rows = sh.rows
        self.total_rows = total_rows

    def flat_values(self):
        """The shard's rows of a flat column whose block payload is its values."""
        parts = [self.blocks[b][0][j * PAGE_ROWS:j * PAGE_ROWS + m.num_values] for (b, j), m in zip(self.pages, self.metas)]
        return np.concatenate(parts) if parts else np.zeros(0)


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
    """This rank's page shard of one C2 column of world x `rows` rows (weak
    scaling: every rank decodes about `rows` rows of the one column), resident
    in HBM twice (two input copies and two output buffers, alternated per
    step so the 256 MiB Infinity Cache cannot serve a step from the previous
    one).  Pages are written by the engine's writer at ratio 1.2, 64 pages per
    writer call (BLOCK_PAGES)."""

    def __init__(self, torch, pa, rows, seed, variant, device, threads, dist=None, world=1, rank=0):
        t0 = time.time()

        def make_block(b, r0, n):
            v = gen_c2(n, seed, variant, r0)
            opts = pa.WriteOptions(default_compress_ratio=1.2, max_page_size=PAGE_ROWS, seed=seed * 1000003 + b)
            chunk, metas = pa.encode_column(v, None, False, opts, n_threads=threads)
            return v, chunk, metas

        self.col = ShardedColumn(pa, dist, world, rank, world * rows, make_block)
        self.encode_s = time.time() - t0
        self.chunk, self.metas = self.col.chunk, self.col.metas
        self.values = self.col.flat_values().astype(np.int32)
        self.col.blocks.clear()
        self.mix = codec_mix(self.chunk, self.metas)
        self.rows = self.col.rows
        self.in_bytes = len(self.chunk)
        self.out_bytes = self.rows * 4
        dev = f"cuda:{device}"
        host = torch.from_numpy(np.frombuffer(self.chunk, dtype=np.uint8).copy())
        self.decs, self.outs = [], []
        for _ in range(2):
            d = pa.ColumnDecoder.for_shard(host.to(dev), self.metas, self.col.shard, np.int32, False)
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


def step_clocks(wall_s: float, kern_ms, step_bytes: int) -> dict:
    """A workload's step time on both clocks: the host wall clock over the
    timed steps (ms_per_step) and the HIP-event span of the same steps per
    step (kernel_ms_per_step), each with the roofline fraction of the
    step's algorithmic bytes on that clock."""
    km = float(np.median(kern_ms))
    return {
        "ms_per_step": round(wall_s * 1e3, 3),
        "kernel_ms_per_step": round(km, 4),
        "step_traffic_GBps": round(step_bytes / (km / 1e3) / 1e9, 1),
        "roofline_frac": round(step_bytes / (km / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
        "roofline_frac_wall": round(step_bytes / wall_s / 1e9 / HBM_PEAK_GBPS, 4),
    }


def timed(torch, dist, wl: Workload, steps: int, warmup: int):
    for k in range(warmup):
        wl.step(k)
    for k in range(warmup, 2):  # (untimed) every rotating buffer decoded once before the check
        wl.step(k)
    torch.cuda.synchronize()
    ok = wl.verify(torch)
    # The timed region: `steps` steps back to back, bracketed by a barrier and
    # a device synchronize (ms_per_step), with a HIP event on the launch
    # stream (the context launches on torch's current stream) before the first
    # and after the last step: their device-clock span / steps is the step's
    # device time.  No event between steps: each one is a barrier on the
    # queue, 3-10 us a step on the device (tools/evgap.py), which no decode
    # pays.
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for k in range(steps):
        wl.step(k)
    e1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    for d in wl.decs:
        d.check()
    kern_ms = [e0.elapsed_time(e1) / steps]
    return t1 - t0, kern_ms, ok


def encode_gpu(torch, pa, rows: int, device: int, threads: int, steps: int) -> dict:
    """Device page encode (sb_encode_column_device): the headline C2 column
    with the writer's adaptive choice at ratio 1.2 (stats, seeded sampler,
    Bitpacking / Dict / RLE cascade on the GPU), the C2 "b12" column with the
    forced Bitpacking codec and ratio None (the sizing + assembly fast path),
    and configs[0]'s Int64 None column: input GB/s per call (values resident
    in HBM; the call includes its page-table scan and the metas read-back),
    checked byte for byte against the host writer with the same options."""
    out = {}
    cases = [("c2_int32_adaptive_ratio1.2", gen_c2(rows, 42, "mix"), dict(default_compress_ratio=1.2, seed=42)),
             ("c2_int32_forced_bitpacking", gen_c2(rows, 4242, "b12"), dict(forced_codec=14)),
             ("c1_int64_none", np.random.default_rng(42).integers(-2**63, 2**63 - 1, 1_000_000, dtype=np.int64), {})]
    for name, v, kw in cases:
        opts = pa.WriteOptions(max_page_size=PAGE_ROWS, **kw)
        tv = torch.from_numpy(v).to(f"cuda:{device}")
        chunk, metas = pa.encode_column_device(tv, None, False, opts)
        t0 = time.perf_counter()
        host, _ = pa.encode_column(v, None, False, opts, n_threads=threads)
        th = time.perf_counter() - t0
        ok = chunk.cpu().numpy().tobytes() == host
        # the C-ABI call itself (pages sized, scanned and written; metas read back), buffers preallocated
        import ctypes

        from pa_amd import _native as N

        phys = pa.read.physical_type(v.dtype)
        cap = N.lib().sb_encode_device_bound(phys, len(v), 0, PAGE_ROWS)
        dout = torch.empty(cap, dtype=torch.uint8, device=tv.device)
        npg = (len(v) + PAGE_ROWS - 1) // PAGE_ROWS
        metas = (N.PageMetaC * npg)()
        olen, nout, copts = ctypes.c_uint64(), ctypes.c_uint64(), opts.c()
        ctx = pa.default_context(device)

        def call():
            st = N.lib().sb_encode_column_device(ctx._h, phys, ctypes.c_void_p(tv.data_ptr()), None, len(v), 0,
                                                 ctypes.byref(copts), PAGE_ROWS, ctypes.c_void_p(dout.data_ptr()),
                                                 cap, ctypes.byref(olen), metas, npg, ctypes.byref(nout))
            assert st == 0, st

        call()
        torch.cuda.synchronize()
        k = max(3, steps // 4)
        t0 = time.perf_counter()
        for _ in range(k):
            call()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / k
        ok &= dout[: olen.value].cpu().numpy().tobytes() == host
        out[name] = {"rows": len(v), "input_GBps": round(v.nbytes / dt / 1e9, 1), "ms_per_call": round(dt * 1e3, 3),
                     "encoded_bytes": len(host), "host_writer_GBps": round(v.nbytes / th / 1e9, 2),
                     "host_threads": threads, "byte_identical_to_host": bool(ok)}
        del tv, chunk, dout
    out["c4_list_int32_adaptive_ratio1.2"] = encode_list_gpu(torch, pa, rows // 2, device, threads, steps)
    out["zstd_size_vs_libzstd3"] = zstd_size(torch, pa, device, threads)
    return out


def encode_list_gpu(torch, pa, rows: int, device: int, threads: int, steps: int) -> dict:
    """Device List encode (sb_encode_list_column_device) of a C4-shaped
    column (List<Int32>, nullable lists and items, lengths in {0, 1, 2},
    ratio 1.2, 8192-row pages): level headers and child values on the GPU,
    byte for byte against the host writer (sb_encode_list_column); input
    GB/s = offsets + child values + both bitmaps per call."""
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 3, rows)
    lv = rng.random(rows) >= 0.1
    lens[~lv] = 0
    offs = np.zeros(rows + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    child = rng.integers(0, 1 << 16, int(offs[-1])).astype(np.int32)
    cv = rng.random(len(child)) >= 0.2
    opts = pa.WriteOptions(default_compress_ratio=1.2, max_page_size=PAGE_ROWS, seed=7)
    t0 = time.perf_counter()
    host, hm = pa.encode_list_column(offs, child, lv, cv, True, True, opts, n_threads=threads)
    th = time.perf_counter() - t0
    dev = lambda a: torch.from_numpy(a).to(f"cuda:{device}")  # noqa: E731
    do, dc, dl, dv = dev(offs), dev(child), dev(lv), dev(cv)
    chunk, dm = pa.encode_list_column_device(do, dc, dl, dv, True, True, opts)
    ok = chunk.cpu().numpy().tobytes() == bytes(host) and [(m.length, m.num_values) for m in dm] == \
        [(m.length, m.num_values) for m in hm]
    torch.cuda.synchronize()
    k = max(3, steps // 4)
    t0 = time.perf_counter()
    for _ in range(k):
        pa.encode_list_column_device(do, dc, dl, dv, True, True, opts)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    nbytes = offs.nbytes + child.nbytes + (rows + 7) // 8 + (len(child) + 7) // 8
    return {"rows": rows, "leaves": int(len(child)), "input_GBps": round(nbytes / dt / 1e9, 1),
            "ms_per_call": round(dt * 1e3, 3), "encoded_bytes": len(host), "host_writer_GBps": round(nbytes / th / 1e9, 2),
            "host_threads": threads, "byte_identical_to_host": bool(ok),
            "call": "pa_amd.encode_list_column_device (bitmaps packed on the device, metas read back)"}


def zstd_size(torch, pa, device: int, threads: int, rows: int = 8 * 1024 * 1024) -> dict:
    """Default-Zstd chunks written on the device (sb_zstdc.h: frames transcoded
    from the wave LZ4 parse) against the host writer's (libzstd level 3, what
    the reference's zstd::bulk::compress level 0 writes, basic.rs:122-135),
    in bytes, on C3's two columns (1024 pages each); LZ4 chunk bytes beside
    them.  Both decode to the same values (tests/test_gpu_encode_adaptive.py)."""
    rng = np.random.default_rng(3)
    f = np.round(rng.standard_normal(rows) * 1e4, 2)
    svals, soffs = decimal_strings(rng.integers(0, 10**6, rows))
    dev = f"cuda:{device}"
    res = {}
    for name in ("c3_float64", "c3_utf8"):
        sizes = {}
        for codec in (2, 1):
            opts = pa.WriteOptions(default_compression=codec, max_page_size=PAGE_ROWS)
            if name == "c3_float64":
                d, _ = pa.encode_column_device(torch.from_numpy(f).to(dev), None, False, opts)
                h, _ = pa.encode_column(f, None, False, opts, n_threads=threads)
            else:
                d, _ = pa.encode_binary_column_device(torch.from_numpy(np.frombuffer(svals, np.uint8).copy()).to(dev),
                                                      torch.from_numpy(soffs).to(dev), None, False, opts,
                                                      physical_type=pa.UTF8)
                h, _ = pa.encode_binary_column(svals, soffs, None, False, opts, physical_type=pa.UTF8,
                                               n_threads=threads)
            sizes[codec] = (int(d.numel()), len(h))
        res[name] = {"device_zstd_bytes": sizes[2][0], "libzstd3_bytes": sizes[2][1],
                     "device_over_libzstd3": round(sizes[2][0] / sizes[2][1], 3), "lz4_bytes": sizes[1][1],
                     "lz4_over_libzstd3": round(sizes[1][1] / sizes[2][1], 3)}
    return res


def cpu_info() -> dict:
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count()
    th = cpu_threads()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": aff,
            "cores_note": f"the 'all cores' leg uses {th} threads: this GPU's CPU allotment on the box "
                          f"(OMP_NUM_THREADS = {os.environ.get('OMP_NUM_THREADS', 'unset')}; {os.cpu_count()} CPUs "
                          f"serve 8 GPUs), not the whole node"}


def cpu_threads() -> int:
    """The box's CPU share: OMP_NUM_THREADS when set (16 per GPU on the pool),
    else all CPUs, at most 16."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env if env > 0 else max(1, min(16, os.cpu_count() or 1))


def time_legs(fn, out_bytes: int, budget_s: float = 4.0) -> dict:
    """fn(threads) decodes the workload once; timed on 1 thread and on the
    box's CPU share, repeated within budget_s per leg -> GB/s of each."""
    res = {}
    for name, th in (("one_thread", 1), ("all_cores", cpu_threads())):
        t0 = time.perf_counter()
        fn(th)
        first = time.perf_counter() - t0
        reps = max(1, min(20, int(budget_s / max(first, 1e-3))))
        t0 = time.perf_counter()
        for _ in range(reps):
            fn(th)
        dt = (time.perf_counter() - t0) / reps
        res[name] = {"GBps": round(out_bytes / dt / 1e9, 3), "threads": th, "s_per_pass": round(dt, 4)}
    return res


def cpu_baseline(wl: Workload) -> dict:
    """The oracle's restatement of read_integer over the headline column:
    compressed pages in host RAM -> values in host RAM, 1 thread and all cores."""
    from oracle import oracle as O

    metas = [(m.length, m.num_values) for m in wl.metas]
    src = np.frombuffer(wl.chunk, np.uint8)
    out = (np.empty(wl.rows, np.int32), np.zeros(wl.rows // 8 + 2, np.uint8))
    v, _ = O.mt_read_column(src, metas, np.int32, False, cpu_threads(), out)
    assert np.array_equal(v[: wl.rows], wl.values), "CPU decode mismatch"
    legs = time_legs(lambda th: O.mt_read_column(src, metas, np.int32, False, th, out), wl.out_bytes)
    allc = legs["all_cores"]
    return {
        "value": allc["GBps"],
        "unit": "GB/s",
        "cores": allc["threads"],
        "kind": "port",
        "sample": f"oracle/ C restatement of read_integer over the full {wl.rows}-row column (compressed pages in "
                  f"host RAM -> values in host RAM), pages sharded over {allc['threads']} threads; the 1-thread leg "
                  f"is the reference's single-threaded shape",
        "one_thread": legs["one_thread"],
        **cpu_info(),
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


class StreamSet:
    """Independent columns decode concurrently (the reference decodes columns
    independently too, read/deserialize.rs:237-253): each column's context
    launches on one of `n` side streams, forked from and joined back into the
    current stream every step, so the HIP events of timed() span all of them.
    mode "torch": torch's pooled side streams; "own": each context on a HIP
    stream of its own (pa.Context.use_own_stream); "prio": torch side streams,
    the last at high priority.  Streams of equal priority may share one
    hardware queue, and then the columns run one after the other: C3 took
    4.46 ms/step on torch streams and 3.96 on its own ones in one process
    (tools/wlstreams.py), 4.0 and 4.5 in the bench's, after other workloads had
    created their streams."""

    def __init__(self, torch, pa, device, n, mode="torch"):
        self.torch = torch
        self.ctxs = [pa.Context(device) for _ in range(n)]
        mode = os.environ.get("SB_BENCH_STREAMS", mode)
        if mode in ("prio", "prio0"):
            # torch side streams, the last one (prio0: the first) at high
            # priority: a queue of its own (priority is a property of the
            # hardware queue), and its column's kernels dispatch first
            hi = 0 if mode == "prio0" else n - 1
            self.streams = [torch.cuda.Stream(device=device, priority=-1 if i == hi else 0) for i in range(n)]
            for c, st in zip(self.ctxs, self.streams):
                c.use_stream(st)
        elif mode == "own":
            # measured slower for C5 (3.39 vs 2.74 ms/step) -- the four
            # streams then run on four hardware queues at once and the LZ4 /
            # Patas units contend with the rest
            self.streams = [c.use_own_stream() for c in self.ctxs]
        else:  # torch's pooled side streams
            self.streams = [torch.cuda.Stream(device=device) for _ in range(n)]
            for c, st in zip(self.ctxs, self.streams):
                c.use_stream(st)
        torch.cuda.synchronize()

    def fork(self):
        cur = self.torch.cuda.current_stream()
        for st in self.streams:
            st.wait_stream(cur)

    def join(self):
        cur = self.torch.cuda.current_stream()
        for st in self.streams:
            cur.wait_stream(st)


def _bits(valid) -> np.ndarray:
    return np.packbits(np.asarray(valid, bool), bitorder="little")


class WorkloadC3:
    """BASELINE.json configs[2]: nullable Float64 + nullable Utf8, LZ4 pages,
    ratio None (always the general codec), 10 % nulls, 8192-row pages; this
    rank's page shard of each of the two columns (world x `rows` rows).  A
    step decodes both shards; two input/output copies rotate."""

    def __init__(self, torch, pa, rows, seed, device, threads, dist=None, world=1, rank=0):
        def opts(b):
            return pa.WriteOptions(default_compression=1, default_compress_ratio=None, max_page_size=PAGE_ROWS,
                                   seed=seed * 1000003 + b)

        def pages(r0, n):
            return [(r0 // PAGE_ROWS + i, min(PAGE_ROWS, n - i * PAGE_ROWS)) for i in range((n + PAGE_ROWS - 1) // PAGE_ROWS)]

        def f_block(b, r0, n):
            f, v = [], []
            for p, m in pages(r0, n):
                rng = page_rng(seed, p)
                f.append(np.round(rng.standard_normal(m) * 1e4, 2))
                v.append(rng.random(m) >= 0.1)
            f, v = np.concatenate(f), np.concatenate(v)
            chunk, metas = pa.encode_column(f, v, True, opts(b), n_threads=threads)
            return (f, v), chunk, metas

        def s_block(b, r0, n):
            ints, v = [], []
            for p, m in pages(r0, n):
                rng = page_rng(seed + 1, p)
                ints.append(rng.integers(0, 10**6, m))
                v.append(rng.random(m) >= 0.1)
            svals, soffs = decimal_strings(np.concatenate(ints))
            v = np.concatenate(v)
            chunk, metas = pa.encode_binary_column(svals, soffs, v, True, opts(b), physical_type=pa.UTF8,
                                                   n_threads=threads)
            return (np.frombuffer(svals, np.uint8), soffs, v), chunk, metas

        self.fcol = ShardedColumn(pa, dist, world, rank, world * rows, f_block)
        self.scol = ShardedColumn(pa, dist, world, rank, world * rows, s_block)
        self.fchunk, self.fmetas = self.fcol.chunk, self.fcol.metas
        self.schunk, self.smetas = self.scol.chunk, self.scol.metas
        # the shards' expected Arrow buffers (offsets shard-local, from 0)
        fv, fm = [], []
        for (b, j), m in zip(self.fcol.pages, self.fcol.metas):
            (f, v), r = self.fcol.blocks[b][0], j * PAGE_ROWS
            fv.append(f[r:r + m.num_values])
            fm.append(v[r:r + m.num_values])
        so, sv, sm, acc = [np.zeros(1, np.int64)], [], [], 0
        for (b, j), m in zip(self.scol.pages, self.scol.metas):
            (vals, offs, v), r = self.scol.blocks[b][0], j * PAGE_ROWS
            o = offs[r:r + m.num_values + 1]
            so.append(o[1:] - o[0] + acc)
            acc += int(o[-1] - o[0])
            sv.append(vals[o[0]:o[-1]])
            sm.append(v[r:r + m.num_values])
        self.fcol.blocks.clear()
        self.scol.blocks.clear()
        f, fvalid = np.concatenate(fv), np.concatenate(fm)
        soffs, svals, svalid = np.concatenate(so), np.concatenate(sv).tobytes(), np.concatenate(sm)
        self.rows = len(f)
        self.srows = len(svalid)
        dev = f"cuda:{device}"
        fh = torch.from_numpy(np.frombuffer(self.fchunk, np.uint8).copy())
        sh = torch.from_numpy(np.frombuffer(self.schunk, np.uint8).copy())
        # Float64 and Utf8 columns on streams of their own: the second column's
        # k_inflate waves take the wave slots the first one's leave as its
        # job queue drains
        self.ss = StreamSet(torch, pa, device, 2, mode="prio0")
        fd, sd = [fh.to(dev) for _ in range(2)], [sh.to(dev) for _ in range(2)]
        torch.cuda.synchronize()
        self.fdec = [pa.ColumnDecoder.for_shard(fd[i], self.fmetas, self.fcol.shard, np.float64, True, ctx=self.ss.ctxs[0])
                     for i in range(2)]
        self.sdec = [pa.BinaryColumnDecoder.for_shard(sd[i], self.smetas, self.scol.shard, pa.UTF8, True,
                                                      ctx=self.ss.ctxs[1]) for i in range(2)]
        self.fout = [d.alloc_outputs() for d in self.fdec]
        self.sout = [d.alloc_outputs() for d in self.sdec]
        # where this shard's Utf8 bytes start in the whole column (the one exchange, setup only)
        self.values_base = pa.shard_base(len(svals), rank) if dist is not None and world > 1 else 0
        self.in_bytes = len(self.fchunk) + len(self.schunk)
        self.out_bytes = self.rows * 8 + (self.rows + 7) // 8 + 4 * (self.srows + 1) + len(svals) + (self.srows + 7) // 8
        self.svals_len = len(svals)
        self.exp = (torch.from_numpy(f.view(np.int64)).to(dev), torch.from_numpy(_bits(fvalid)).to(dev),
                    torch.from_numpy(soffs.astype(np.int32)).to(dev), torch.from_numpy(np.frombuffer(svals, np.uint8).copy()).to(dev),
                    torch.from_numpy(_bits(svalid)).to(dev))
        torch.cuda.synchronize()

    def step(self, k):
        self.ss.fork()
        self.fdec[k & 1].decode_async(*self.fout[k & 1])
        self.sdec[k & 1].decode_async(*self.sout[k & 1])
        self.ss.join()

    def verify(self, torch) -> bool:
        ok = True
        nb, snb = (self.rows + 7) // 8, (self.srows + 7) // 8
        for i in range(2):
            self.fdec[i].check()
            self.sdec[i].check()
            fv, fm = self.fout[i]
            so, sv, sm = self.sout[i]
            ok &= bool(torch.equal(fv[: self.rows], self.exp[0]))
            ok &= bool(torch.equal(fm[:nb], self.exp[1]))
            ok &= bool(torch.equal(so, self.exp[2]))
            ok &= bool(torch.equal(sv[: self.exp[3].numel()], self.exp[3]))
            ok &= bool(torch.equal(sm[:snb], self.exp[4]))
        return ok

    @property
    def decs(self):
        return self.fdec + self.sdec

    def cpu_baseline(self) -> dict:
        """read_double + read_binary of both columns on the host (LZ4 through
        the system liblz4, as basic.rs:87-91), 1 thread and all cores."""
        from oracle import oracle as O

        fm = [(m.length, m.num_values) for m in self.fmetas]
        sm = [(m.length, m.num_values) for m in self.smetas]
        fsrc, ssrc = np.frombuffer(self.fchunk, np.uint8), np.frombuffer(self.schunk, np.uint8)
        n, sn = self.rows, self.srows
        fo = (np.empty(n, np.float64), np.zeros(n // 8 + 2, np.uint8))
        so = (np.empty(sn + 1, np.int32), np.empty(self.svals_len + 16, np.uint8), np.zeros(sn // 8 + 2, np.uint8))

        def run(th):
            O.mt_read_column(fsrc, fm, np.float64, True, th, fo)
            O.mt_read_binary_column(ssrc, sm, True, 4, th, self.svals_len + 16, so)

        run(cpu_threads())
        # the GPU's Arrow buffers against the CPU decoder's, byte for byte (values under nulls included)
        nb, snb = (n + 7) // 8, (sn + 7) // 8
        fv, fm_ = self.fout[0]
        go, gv, gm = self.sout[0]
        ok = fv.cpu().numpy().view(np.float64)[:n].tobytes() == fo[0].tobytes()
        ok &= fm_.cpu().numpy()[:nb].tobytes() == fo[1][:nb].tobytes()
        ok &= go.cpu().numpy().tobytes() == so[0].tobytes()
        ok &= gv.cpu().numpy()[: self.svals_len].tobytes() == so[1][: self.svals_len].tobytes()
        ok &= gm.cpu().numpy()[:snb].tobytes() == so[2][:snb].tobytes()
        legs = time_legs(run, self.out_bytes)
        return {"value": legs["all_cores"]["GBps"], "unit": "GB/s", "cores": legs["all_cores"]["threads"],
                "kind": "port", "one_thread": legs["one_thread"], "gpu_bit_exact_vs_cpu": bool(ok),
                "sample": "oracle/ read_double + read_binary of both full columns, LZ4 via the system liblz4"}


class WorkloadC4:
    """BASELINE.json configs[3]: List<Int32>, nullable lists (10 %) of
    nullable items (20 %), lengths uniform in {0, 1, 2} (tests/it/io.rs:399-415
    shape), items uniform in [0, 2^16), adaptive ratio 1.2, 8192-row pages;
    this rank's page shard of one column of world x `rows` outer rows (the
    configs' "pages sharded across GPUs").  A step = sizing pass + level
    decode (offsets, both bitmaps) + values, on the shard."""

    def __init__(self, torch, pa, rows, seed, device, threads, dist=None, world=1, rank=0):
        def l_block(b, r0, n):
            lens, lvs, childs, cvs = [], [], [], []
            for i in range((n + PAGE_ROWS - 1) // PAGE_ROWS):
                m = min(PAGE_ROWS, n - i * PAGE_ROWS)
                rng = page_rng(seed, r0 // PAGE_ROWS + i)
                ln = rng.integers(0, 3, m)
                lv = rng.random(m) >= 0.1
                ln[~lv] = 0
                V = int(ln.sum())
                lens.append(ln)
                lvs.append(lv)
                childs.append(rng.integers(0, 1 << 16, V).astype(np.int32))
                cvs.append(rng.random(V) >= 0.2)
            ln = np.concatenate(lens)
            offs = np.zeros(n + 1, np.int64)
            np.cumsum(ln, out=offs[1:])
            payload = (offs, np.concatenate(childs), np.concatenate(lvs), np.concatenate(cvs))
            opts = pa.WriteOptions(default_compress_ratio=1.2, max_page_size=PAGE_ROWS, seed=seed * 1000003 + b)
            chunk, metas = pa.encode_list_column(*payload, True, True, opts, n_threads=threads)
            return payload, chunk, metas

        self.col = ShardedColumn(pa, dist, world, rank, world * rows, l_block)
        self.chunk, self.metas = self.col.chunk, self.col.metas
        oo, lvv, cc, cvv, acc = [np.zeros(1, np.int64)], [], [], [], 0
        for b, j in self.col.pages:
            offs, child, lv, cv = self.col.blocks[b][0]
            r = j * PAGE_ROWS
            o = offs[r:min(r + PAGE_ROWS, len(offs) - 1) + 1]
            oo.append(o[1:] - o[0] + acc)
            acc += int(o[-1] - o[0])
            lvv.append(lv[r:r + len(o) - 1])
            cc.append(child[o[0]:o[-1]])
            cvv.append(cv[o[0]:o[-1]])
        self.col.blocks.clear()
        offs, lv, child, cv = np.concatenate(oo), np.concatenate(lvv), np.concatenate(cc), np.concatenate(cvv)
        self.rows, V = len(lv), len(child)
        self.mix = {}
        dev = f"cuda:{device}"
        h = torch.from_numpy(np.frombuffer(self.chunk, np.uint8).copy())
        self.decs = [pa.ListColumnDecoder.for_shard(h.to(dev), self.metas, self.col.shard, np.int32, True, True)
                     for _ in range(2)]
        self.outs = [d.alloc_outputs() for d in self.decs]
        self.leaves = V
        # where this shard's leaves start in the whole column (the one exchange, setup only)
        self.leaf_base = pa.shard_base(V, rank) if dist is not None and world > 1 else 0
        self.in_bytes = len(self.chunk)
        self.out_bytes = 4 * (self.rows + 1) + (self.rows + 7) // 8 + 4 * V + (V + 7) // 8
        self.exp = (torch.from_numpy(offs.astype(np.int32)).to(dev), torch.from_numpy(_bits(lv)).to(dev),
                    torch.from_numpy(child).to(dev), torch.from_numpy(_bits(cv)).to(dev),
                    torch.from_numpy(cv).to(dev))
        torch.cuda.synchronize()

    def step(self, k):
        self.decs[k & 1].decode_async(*self.outs[k & 1])

    def cpu_baseline(self) -> dict:
        """read_validity_nested + create_list + read_integer over every page on
        the host (the oracle), 1 thread and all cores."""
        from oracle import oracle as O

        m = [(x.length, x.num_values) for x in self.metas]
        src = np.frombuffer(self.chunk, np.uint8)
        lev = sum(x.num_values for x in self.metas)
        out = (np.empty(lev + 2, np.int64), np.zeros(lev // 8 + 2, np.uint8), np.empty(lev + 1, np.int32),
               np.zeros(lev // 8 + 2, np.uint8))
        r = O.mt_read_list_column(src, m, np.int32, True, True, cpu_threads(), out)
        # the GPU's buffers against the CPU decoder's, byte for byte (values under null items included)
        o, lv, v, fv = self.outs[0]
        R, V = self.rows, self.leaves
        ok = r[4] == R and r[5] == V
        ok &= np.array_equal(o.cpu().numpy().astype(np.int64), out[0][: R + 1])
        ok &= lv.cpu().numpy()[: (R + 7) // 8].tobytes() == out[1][: (R + 7) // 8].tobytes()
        ok &= v.cpu().numpy()[:V].tobytes() == out[2][:V].tobytes()
        ok &= fv.cpu().numpy()[: (V + 7) // 8].tobytes() == out[3][: (V + 7) // 8].tobytes()
        legs = time_legs(lambda th: O.mt_read_list_column(src, m, np.int32, True, True, th, out), self.out_bytes)
        return {"value": legs["all_cores"]["GBps"], "unit": "GB/s", "cores": legs["all_cores"]["threads"],
                "kind": "port", "one_thread": legs["one_thread"], "gpu_bit_exact_vs_cpu": bool(ok),
                "sample": "oracle/ nested page reader over every page of the column"}

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


def page_codecs(chunk: bytes, metas, nullable: bool) -> dict:
    """Codec byte of every page's (first) value stream, after the validity prefix."""
    mix, pos = {}, 0
    for m in metas:
        q = pos + (4 + int.from_bytes(chunk[pos:pos + 4], "little") if nullable else 0)
        c = chunk[q] if q < pos + m.length else -1
        mix[c] = mix.get(c, 0) + 1
        pos += m.length
    return mix


class WorkloadC5:
    """BASELINE.json configs[4]: a 64-column table of
    `rows` rows -- 16 Int32, 16 Int64, 8 Float64, 8 Utf8, 8 Boolean, 8 UInt32
    -- in 8192-row pages at default_compress_ratio 2.0 (tests/it/io.rs:433),
    each column shaped for a codec of the adaptive cascade (the LZ4 / None
    columns written with that default codec and no ratio); every fourth
    fixed-width or Boolean column nullable (10 % nulls).  Every column is
    encoded on the GPU from values resident in HBM (sb_encode_column_device /
    sb_encode_binary_column_device; timed) and checked byte for byte against
    the host C++ writer's chunk (timed on the host threads for comparison).
    A step decodes all 64 device-encoded columns over 4 streams; each column
    is checked against its source values."""

    I32 = ["bp4", "bp8", "bp12", "bp16", "bp20", "runs", "runs", "one", "one", "freq", "freq", "dict", "dict",
           "sorted", "sorted", "sorted"]
    I64 = ["runs"] * 4 + ["dict"] * 4 + ["freq"] * 4 + ["none"] * 4
    F64 = ["slow", "patas", "patas", "dict", "runs", "runs", "lz4", "lz4"]
    STR = ["dict", "dict", "freq", "freq", "one", "one", "lz4", "lz4"]
    BOOL = ["runs", "runs", "runs", "one", "one", "none", "none", "none"]
    U32 = ["bp6", "bp10", "bp14", "bp18", "sorted", "sorted", "sorted", "sorted"]

    @staticmethod
    def _values(dt, kind, n, rng):
        if kind.startswith("bp"):
            return rng.integers(0, 1 << int(kind[2:]), n).astype(dt)
        if kind == "runs":
            if dt == np.bool_:
                return np.repeat(rng.random(n // 1000 + 1) > 0.5, 1000)[:n]
            return np.repeat(rng.integers(0, 2**31, n // 200 + 1), 200)[:n].astype(dt)
        if kind == "one":
            return np.ones(n, dt) if dt == np.bool_ else np.full(n, 7, dt)
        if kind == "freq":
            return np.where(rng.random(n) < 0.95, 300, rng.integers(0, 10**6, n)).astype(dt)
        if kind == "dict":
            pool = rng.integers(0, 2**31, 500)
            v = pool[rng.integers(0, 500, n)]
            return (v.astype(np.float64) / 7.0).astype(dt) if dt == np.float64 else v.astype(dt)
        if kind == "sorted":  # sorted within each page (the stats are per page): DeltaBitpacking
            inc = rng.integers(0, 100, n)
            c = np.cumsum(inc)
            start = np.repeat(c[::PAGE_ROWS] - inc[::PAGE_ROWS], PAGE_ROWS)[:n]
            return (c - start).astype(dt)
        if kind == "slow":  # slowly varying with repeats (Dict / RLE friendly)
            return (1000.0 + np.cumsum(rng.integers(-1, 2, n)) * 0.5).astype(dt)
        if kind == "patas":  # each value thrice, a small random walk: too many distinct values for Dict,
            # runs of 3 too short for RLE, equal / near neighbours for Patas (double/patas.rs:37-105)
            walk = 1000.0 + np.cumsum(rng.integers(1, 64, n // 3 + 1)) * 2.0**-20
            return np.repeat(walk, 3)[:n].astype(dt)
        if dt == np.bool_:  # "none"
            return rng.random(n) > 0.5
        if dt == np.float64:  # "lz4"
            return np.round(rng.standard_normal(n) * 1e4, 2)
        return rng.integers(-2**62, 2**62, n).astype(dt)  # "none": incompressible

    @staticmethod
    def _strings(kind, n, rng):
        if kind == "dict":
            pool = [f"category-{i:04d}".encode() for i in range(200)]
            s = [pool[i] for i in rng.integers(0, 200, n)]
        elif kind == "freq":
            s = [b"common-value" if r < 0.95 else str(x).encode() for r, x in zip(rng.random(n), rng.integers(0, 10**6, n))]
        elif kind == "one":
            s = [b"constant"] * n
        else:
            return decimal_strings(rng.integers(0, 10**6, n))
        offs = np.zeros(n + 1, np.int64)
        np.cumsum([len(x) for x in s], out=offs[1:])
        return b"".join(s), offs

    @classmethod
    def specs(cls):
        """(dtype | "utf8", value kind) of the table's 64 columns, in order."""
        return ([(np.int32, k) for k in cls.I32] + [(np.int64, k) for k in cls.I64] +
                [(np.float64, k) for k in cls.F64] + [("utf8", k) for k in cls.STR] +
                [(np.bool_, k) for k in cls.BOOL] + [(np.uint32, k) for k in cls.U32])

    @staticmethod
    def rank_columns(n_columns, world, rank):
        """The table's columns round-robin over the ranks:
        this rank builds and decodes columns ci with ci % world == rank."""
        return [ci for ci in range(n_columns) if ci % world == rank]

    @classmethod
    def host_column(cls, pa, dt, kind, ci, rows, seed, threads):
        """Column ci's source values and its host-writer chunk ->
        (values | (bytes, offsets), validity | None, nullable, opts, chunk, metas, host encode seconds)."""
        rng = np.random.default_rng([seed, ci])  # each column its own generator
        nullable = dt != "utf8" and ci % 4 == 3
        valid = (rng.random(rows) >= 0.1) if nullable else None
        basic = kind in ("lz4", "none")
        opts = pa.WriteOptions(default_compression=1 if kind == "lz4" else 0,
                               default_compress_ratio=None if basic else 2.0, max_page_size=PAGE_ROWS, seed=seed + ci)
        if dt == "utf8":
            svals, soffs = cls._strings(kind, rows, rng)
            t0 = time.perf_counter()
            chunk, metas = pa.encode_binary_column(svals, soffs, None, False, opts, physical_type=pa.UTF8,
                                                   n_threads=threads)
            return (svals, soffs), None, False, opts, chunk, metas, time.perf_counter() - t0
        v = cls._values(dt, kind, rows, rng)
        t0 = time.perf_counter()
        chunk, metas = pa.encode_column(v, valid, nullable, opts, n_threads=threads)
        return v, valid, nullable, opts, chunk, metas, time.perf_counter() - t0

    def __init__(self, torch, pa, rows, seed, device, threads, world=1, rank=0):
        self.rows = rows
        self.threads = threads
        dev = f"cuda:{device}"
        specs = self.specs()
        self.n_columns = len(specs)
        self.col_ids = self.rank_columns(len(specs), world, rank)
        specs = [specs[ci] for ci in self.col_ids]
        self.cols = []
        self.host = []  # (dt, chunk, metas, nullable, values_len) for the CPU baseline
        self.encode_s = 0.0
        self.in_bytes = self.out_bytes = self.raw_bytes = 0
        self.mix = {}
        names = {0: "none", 1: "lz4", 2: "zstd", 3: "snappy", 10: "rle", 11: "dict", 12: "one_value", 13: "freq",
                 14: "bitpacking", 15: "delta_bitpacking", 16: "patas"}
        nb = (rows + 7) // 8
        self.ss = StreamSet(torch, pa, device, int(os.environ.get("SB_C5_STREAMS", "4")))
        enc = []  # device encode inputs: (dt, opts, nullable, device tensors)
        for ci, (dt, kind) in zip(self.col_ids, specs):
            v, valid, nullable, opts, chunk, metas, enc_s = self.host_column(pa, dt, kind, ci, rows, seed, threads)
            self.encode_s += enc_s
            if dt == "utf8":
                svals, soffs = v
                raw = len(svals) + 4 * (rows + 1)
                exp = (torch.from_numpy(soffs.astype(np.int32)).to(dev),
                       torch.from_numpy(np.frombuffer(svals, np.uint8).copy()).to(dev))
                enc.append((dt, opts, False, (exp[1], torch.from_numpy(soffs).to(dev), None)))
                self.host.append((dt, chunk, metas, False, len(svals)))
            else:
                raw = nb if dt == np.bool_ else v.nbytes
                tv = torch.from_numpy(v).to(dev)
                ev = tv if dt == np.bool_ else tv.view(torch.uint8)
                tvalid = None if valid is None else torch.from_numpy(valid).to(dev)
                exp = (ev, tvalid)
                enc.append((dt, opts, nullable, (tv, tvalid)))
                self.host.append((dt, chunk, metas, nullable, 0))
            for c, k in page_codecs(chunk, metas, nullable).items():
                self.mix[names.get(c, str(c))] = self.mix.get(names.get(c, str(c)), 0) + k
            self.raw_bytes += raw
            self.out_bytes += raw + (nb if nullable else 0)
            self.in_bytes += len(chunk)
            self.cols.append([dt, None, None, exp, chunk, metas, nullable])
        torch.cuda.synchronize()
        # device encode of every column (values in HBM): a warm-up pass (context
        # scratch), then a timed pass; byte-identical to the host writer
        self.encode_gpu_s, self.byte_identical = self._encode_device(torch, pa, enc, device)
        # decoders over the device-encoded chunks: the fixed-width and Boolean
        # leaves of one type and nullability as one plan each
        # (pa_amd.ColumnGroupDecoder: their chunks back to back, as in a file),
        # the Utf8 leaves one plan each; then longest first onto the least
        # loaded of the 4 streams (each unit's cost from one timed decode)
        groups = {}
        for ci, col in enumerate(self.cols):
            if col[0] != "utf8":
                groups.setdefault((np.dtype(col[0]).str, col[6]), []).append(ci)
        self.units = []
        for cis in groups.values():
            g = pa.ColumnGroupDecoder([(self.dev_chunks[ci], self.cols[ci][5]) for ci in cis], self.cols[cis[0]][0],
                                      self.cols[cis[0]][6], ctx=self.ss.ctxs[0])
            outs = g.alloc_outputs()
            for i, ci in enumerate(cis):
                self.cols[ci][1], self.cols[ci][2] = g, g.column(i, *outs)
            self.units.append([g, outs])
        for ci, col in enumerate(self.cols):
            if col[0] == "utf8":
                dec = pa.BinaryColumnDecoder(self.dev_chunks[ci], col[5], pa.UTF8, False, ctx=self.ss.ctxs[0])
                col[1], col[2] = dec, dec.alloc_outputs()
                self.units.append([dec, col[2]])
        del self.dev_chunks
        cost = []
        for u in self.units:
            u[0].decode_async(*u[1])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            u[0].decode_async(*u[1])
            torch.cuda.synchronize()
            cost.append(time.perf_counter() - t0)
        load = [0.0] * len(self.ss.ctxs)
        order = sorted(range(len(self.units)), key=lambda i: -cost[i])
        for i in order:
            s_ = min(range(len(load)), key=lambda j: load[j])
            load[s_] += cost[i]
            self.units[i][0].ctx = self.ss.ctxs[s_]
        self.units = [self.units[i] for i in order]
        self.n_launch_units = len(self.units)
        torch.cuda.synchronize()

    def _encode_device(self, torch, pa, enc, device):
        same = True
        best = None
        for rep in range(3):
            chunks = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cols = [pa.DeviceColumn(t[0], None, False, opts, t[1], pa.UTF8) if dt == "utf8" else
                    pa.DeviceColumn(t[0], t[1], nullable, opts) for dt, opts, nullable, t in enc]
            chunks = pa.encode_table_device(cols, n_streams=int(os.environ.get("SB_ENC_STREAMS", "4")), device=device)
            torch.cuda.synchronize()
            dt_s = time.perf_counter() - t0
            if rep:
                best = dt_s if best is None else min(best, dt_s)
        for (c, m), col in zip(chunks, self.cols):
            same &= c.cpu().numpy().tobytes() == col[4]
            same &= [(x.length, x.num_values) for x in m] == [(x.length, x.num_values) for x in col[5]]
        self.dev_chunks = [c for c, _ in chunks]
        return best, bool(same)

    def cpu_baseline(self) -> dict:
        """Every column's reader on the host (read_integer / read_double /
        read_boolean / read_binary restated by the oracle), 1 thread and all cores."""
        from oracle import oracle as O

        n = self.rows
        jobs, cpu_outs = [], []
        for dt, chunk, metas, nullable, vlen in self.host:
            m = [(x.length, x.num_values) for x in metas]
            src = np.frombuffer(chunk, np.uint8)
            if dt == "utf8":
                out = (np.empty(n + 1, np.int32), np.empty(vlen + 16, np.uint8), np.zeros(n // 8 + 2, np.uint8))
                jobs.append(lambda th, src=src, m=m, out=out, vlen=vlen:
                            O.mt_read_binary_column(src, m, False, 4, th, vlen + 16, out))
            elif dt == np.bool_:
                out = (np.zeros(n // 8 + 2, np.uint8), np.zeros(n // 8 + 2, np.uint8))
                jobs.append(lambda th, src=src, m=m, out=out, nl=nullable: O.mt_read_bool_column(src, m, nl, th, out))
            else:
                out = (np.empty(n, dt), np.zeros(n // 8 + 2, np.uint8))
                jobs.append(lambda th, src=src, m=m, out=out, nl=nullable, dt=dt:
                            O.mt_read_column(src, m, dt, nl, th, out))
            cpu_outs.append(out)

        def run(th):
            for j in jobs:
                j(th)

        run(cpu_threads())
        # every column's GPU buffers against the CPU decoder's, byte for byte (values under nulls included)
        ok = True
        nb = (n + 7) // 8
        for col, cpu, host in zip(self.cols, cpu_outs, self.host):
            dt, outs = col[0], col[2]
            if dt == "utf8":
                vlen = host[4]
                ok &= outs[0].cpu().numpy().tobytes() == cpu[0].tobytes()
                ok &= outs[1].cpu().numpy()[:vlen].tobytes() == cpu[1][:vlen].tobytes()
            elif dt == np.bool_:
                ok &= outs[0].cpu().numpy()[:nb].tobytes() == cpu[0][:nb].tobytes()
                if col[6]:
                    ok &= outs[1].cpu().numpy()[:nb].tobytes() == cpu[1][:nb].tobytes()
            else:
                ok &= outs[0].cpu().numpy().view(np.uint8)[: n * np.dtype(dt).itemsize].tobytes() == cpu[0].tobytes()
                if col[6]:
                    ok &= outs[1].cpu().numpy()[:nb].tobytes() == cpu[1][:nb].tobytes()
        legs = time_legs(run, self.out_bytes, budget_s=3.0)
        return {"value": legs["all_cores"]["GBps"], "unit": "GB/s", "cores": legs["all_cores"]["threads"],
                "kind": "port", "one_thread": legs["one_thread"], "gpu_bit_exact_vs_cpu": bool(ok),
                "sample": "oracle/ readers over all 64 columns (compressed pages in host RAM -> Arrow buffers in host "
                          "RAM), each column's pages sharded over the threads"}

    @property
    def decs(self):
        return [u[0] for u in self.units]

    def step(self, k):
        self.ss.fork()
        for dec, outs in self.units:
            dec.decode_async(*outs)
        self.ss.join()

    def verify(self, torch) -> bool:
        ok = True
        n = self.rows
        for dt, dec, outs, exp, _, _, _ in self.cols:
            dec.check()
            if dt == "utf8":
                o, v, _ = outs
                ok &= bool(torch.equal(o, exp[0])) and bool(torch.equal(v[: exp[1].numel()], exp[1]))
                continue
            vals, bm = outs
            ev, valid = exp
            if dt == np.bool_:
                bits = ((vals[: (n + 7) // 8].unsqueeze(1) >> torch.arange(8, device=vals.device, dtype=torch.uint8)) & 1)
                got = bits.reshape(-1)[:n].bool()
            else:
                got = vals.view(torch.uint8)[: ev.numel()]
                if valid is not None:  # compare the valid rows only (values under nulls are the writer's choice)
                    w = np.dtype(dt).itemsize
                    got, ev = got.view(-1, w)[valid], ev.view(-1, w)[valid]
                ok &= bool(torch.equal(got, ev))
                continue
            if valid is not None:
                got, ev = got[valid], ev[valid]
            ok &= bool(torch.equal(got, ev))
        return ok


TRAFFIC_FILE = "r06c_pmc_traffic.json"  # tools/pmc_traffic.sh -> tools/publish_traffic.py


def load_traffic(workload: str):
    """This round's measured HBM bytes per step for `workload` (FETCH_SIZE /
    WRITE_SIZE passes, calibrated correction, the commit they measured), or
    None when the profile is absent."""
    p = os.path.join(ROOT, "profiles", TRAFFIC_FILE)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        t = json.load(f).get(workload)
    if t:
        t = {k: v for k, v in t.items() if k != "kernels"}
    return t


def file_pipeline(torch, pa, wl, device, steps) -> dict:
    """The C2 column read end to end (never the headline
    value): the chunk written to a strawboat file (footer + IPC schema), then
    per step read_meta (footer pre-read), the pinned double-buffered pread ->
    H2D upload (sb_file_upload) into the planned chunk buffer and the decode.
    The file sits in the host page cache, so this is host memory -> PCIe ->
    HBM -> Arrow, not disk."""
    import tempfile

    import pyarrow as pyarrow

    schema = pyarrow.schema([pyarrow.field("c2", pyarrow.int32(), False)]).serialize().to_pybytes()[8:]
    fd, path = tempfile.mkstemp(suffix=".sb", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        with os.fdopen(fd, "wb") as fh:
            fh.write(pa.assemble_file([(wl.chunk, wl.metas)], schema))
        dec, (v, m) = wl.decs[0], wl.outs[0]
        with pa.StrawboatFile(path) as f:  # warm-up: staging buffers, page cache
            f.upload(0, out=dec.chunk)
            dec.decode_async(v, m)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            with pa.StrawboatFile(path) as f:
                f.upload(0, out=dec.chunk)
                dec.decode_async(v, m)
            torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / steps
        with pa.StrawboatFile(path) as f:
            t0 = time.perf_counter()
            for _ in range(steps):
                f.upload(0, out=dec.chunk)
            torch.cuda.synchronize()
            t_up = (time.perf_counter() - t0) / steps
        ok = bool(torch.equal(v, wl.expect))
    finally:
        os.unlink(path)
    return {"file_to_arrow_GBps": round(wl.out_bytes / t_all / 1e9, 2), "ms_per_step": round(t_all * 1e3, 3),
            "h2d_upload_GBps": round(wl.in_bytes / t_up / 1e9, 2), "upload_ms": round(t_up * 1e3, 3),
            "file_bytes": wl.in_bytes, "bit_exact": ok,
            "path": "footer pre-read + IPC schema parse, 2 x 16 MiB pinned buffers (8 pread threads) -> H2D on a "
                    "copy stream, decode on the context stream; file in the page cache (/dev/shm)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-b12", action="store_true", help="skip the all-bitpack b=12 variant")
    ap.add_argument("--no-hard", action="store_true", help="skip the harder C2 mix (b 12..24, RLE runs of 2-3)")
    ap.add_argument("--no-c3", action="store_true", help="skip the config-3 (Float64 + Utf8, LZ4) workload")
    ap.add_argument("--c3-rows", type=int, default=100_000_000)
    ap.add_argument("--no-c4", action="store_true", help="skip the config-4 (List<Int32>) workload")
    ap.add_argument("--c4-rows", type=int, default=50_000_000)
    ap.add_argument("--no-c5", action="store_true", help="skip the config-5 (64-column mixed table) workload")
    ap.add_argument("--no-encode", action="store_true", help="skip the device page encode measurement")
    ap.add_argument("--encode-rows", type=int, default=100_000_000)
    ap.add_argument("--c5-rows", type=int, default=8_388_608)
    ap.add_argument("--no-file", action="store_true", help="skip the file -> HBM -> Arrow pipeline measurement")
    args = ap.parse_args()

    import torch

    import pa_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box: SB_BENCH_BACKEND=gloo puts
    # every rank on cuda:0 (RCCL needs one GPU per rank)
    backend = os.environ.get("SB_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as tdist

        if backend == "gloo":
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        dist = tdist
    threads = max(1, min(16, (os.cpu_count() or 8) // max(world, 1)))
    pa_amd.default_context(local)
    do_cpu = world == 1 and not args.no_cpu  # CPU baselines on rank 0 at N=1 only

    def reduce(x: float, op) -> float:  # (the timing barrier's companions: max wall, summed bytes)
        if not dist:
            return x
        t = torch.tensor([x], device="cpu" if backend == "gloo" else f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return float(t[0])

    MAX = dist.ReduceOp.MAX if dist else None
    SUM = dist.ReduceOp.SUM if dist else None
    # one C2 column of world x rows rows; each rank decodes its shard_pages range (for_shard)
    wl = Workload(torch, pa_amd, args.rows, 42, "mix", local, threads, dist, world, rank)
    wall, kern_ms, ok = timed(torch, dist, wl, args.steps, args.warmup)
    wall_max, any_bad = reduce(wall, MAX), reduce(0.0 if ok else 1.0, MAX) > 0
    kavg = float(np.median(kern_ms))
    achieved = (wl.in_bytes + wl.out_bytes) / (kavg / 1e3) / 1e9
    total_out = reduce(float(wl.out_bytes), SUM)
    value = total_out * args.steps / wall_max / 1e9

    extra = {}
    if not args.no_file and world == 1:
        extra["c2_file_pipeline"] = file_pipeline(torch, pa_amd, wl, local, max(3, args.steps // 4))
    if not args.no_hard:
        wlh = Workload(torch, pa_amd, args.rows, 4343, "hard", local, threads, dist, world, rank)
        wh, kh, okh = timed(torch, dist, wlh, args.steps, args.warmup)
        khavg = float(np.median(kh))
        ah = (wlh.in_bytes + wlh.out_bytes) / (khavg / 1e3) / 1e9
        extra["c2_hard_mix"] = {
            "decoded_GBps": round(reduce(float(wlh.out_bytes), SUM) * args.steps / reduce(wh, MAX) / 1e9, 1),
            "kernel_ms": round(khavg, 4),
            "kernel_traffic_GBps": round(ah, 1),
            "roofline_frac": round(ah / HBM_PEAK_GBPS, 4),
            "codec_mix": wlh.mix,
            "compressed_bytes": wlh.in_bytes,
            "traffic": load_traffic("c2_hard_mix"),
            "bit_exact": bool(okh),
        }
        del wlh
    if not args.no_b12:
        wl12 = Workload(torch, pa_amd, args.rows, 4242, "b12", local, threads, dist, world, rank)
        w12, k12, ok12 = timed(torch, dist, wl12, args.steps, args.warmup)
        k12avg = float(np.median(k12))
        a12 = (wl12.in_bytes + wl12.out_bytes) / (k12avg / 1e3) / 1e9
        extra["bitpack_b12"] = {
            "decoded_GBps": round(reduce(float(wl12.out_bytes), SUM) * args.steps / reduce(w12, MAX) / 1e9, 1),
            "kernel_ms": round(k12avg, 4),
            "kernel_traffic_GBps": round(a12, 1),
            "roofline_frac": round(a12 / HBM_PEAK_GBPS, 4),
            "compressed_bytes": wl12.in_bytes,
            "bit_exact": bool(ok12),
        }
        del wl12

    if not args.no_c3:
        wl3 = WorkloadC3(torch, pa_amd, args.c3_rows, 77, local, threads, dist, world, rank)
        steps3 = max(3, args.steps // 4)
        w3, k3, ok3 = timed(torch, dist, wl3, steps3, args.warmup)
        w3m = reduce(w3, MAX)
        extra["c3_f64_utf8_lz4_nullable"] = {
            "rows_per_gpu": wl3.rows,
            "decoded_GBps": round(reduce(float(wl3.out_bytes), SUM) * steps3 / w3m / 1e9, 1),
            **step_clocks(w3m / steps3, k3, wl3.in_bytes + wl3.out_bytes),
            "compressed_bytes_per_gpu": wl3.in_bytes,
            "decoded_bytes_per_gpu": wl3.out_bytes,
            "bit_exact": bool(ok3),
            "parallelism": f"page-shard x{world} of each column (shard_pages / for_shard); Utf8 values base "
                           f"{wl3.values_base} from the all-gathered shard sizes",
            "traffic": load_traffic("c3_f64_utf8_lz4_nullable"),
            "kernels": "Float64: k_decode_staged<8,true> (validity + LZ4 job list) + k_inflate (values); "
                       "Utf8: k_bin_light + k_inflate (offsets rebased + values) + k_bin_light_out",
        }
        if do_cpu:
            extra["c3_f64_utf8_lz4_nullable"]["cpu_baseline"] = wl3.cpu_baseline()
        del wl3

    if not args.no_c4:
        wl4 = WorkloadC4(torch, pa_amd, args.c4_rows, 99, local, threads, dist, world, rank)
        steps4 = max(3, 2 * args.steps)  # 0.15 ms steps: the timed region's fixed costs spread over more of them
        w4, k4, ok4 = timed(torch, dist, wl4, steps4, args.warmup)
        w4m = reduce(w4, MAX)
        extra["c4_list_int32_nested"] = {
            "rows_per_gpu": wl4.rows,
            "leaves_per_gpu": wl4.leaves,
            "pages_per_gpu": len(wl4.metas),
            "decoded_GBps": round(reduce(float(wl4.out_bytes), SUM) * steps4 / w4m / 1e9, 1),
            **step_clocks(w4m / steps4, k4, wl4.in_bytes + wl4.out_bytes),
            "compressed_bytes_per_gpu": wl4.in_bytes,
            "decoded_bytes_per_gpu": wl4.out_bytes,
            "bit_exact": bool(ok4),
            "parallelism": f"page-shard x{world} of one column (shard_pages / for_shard); leaf base {wl4.leaf_base} "
                           f"from the all-gathered leaf counts",
            "traffic": load_traffic("c4_list_int32_nested"),
            "kernels": "k_list_bases + k_list_levels + k_decode_staged<4,false>",
        }
        if do_cpu:
            extra["c4_list_int32_nested"]["cpu_baseline"] = wl4.cpu_baseline()
        del wl4

    if not args.no_c5:
        wl5 = WorkloadC5(torch, pa_amd, args.c5_rows, 555, local, threads, world, rank)
        steps5 = max(3, args.steps // 4)
        w5, k5, ok5 = timed(torch, dist, wl5, steps5, args.warmup)
        w5m = reduce(w5, MAX)
        extra["c5_mixed_64col"] = {
            "rows": args.c5_rows,
            "columns": wl5.n_columns,
            "columns_this_rank": len(wl5.cols),
            "decoded_GBps": round(reduce(float(wl5.out_bytes), SUM) * steps5 / w5m / 1e9, 1),
            **step_clocks(w5m / steps5, k5, wl5.in_bytes + wl5.out_bytes),
            "compressed_bytes_this_rank": wl5.in_bytes,
            "decoded_bytes_this_rank": wl5.out_bytes,
            "codec_mix_pages": wl5.mix,
            "encode_gpu_GBps": round(reduce(float(wl5.raw_bytes), SUM) / reduce(wl5.encode_gpu_s, MAX) / 1e9, 1),
            "encode_gpu_ms": round(reduce(wl5.encode_gpu_s, MAX) * 1e3, 2),
            "encode_byte_identical": wl5.byte_identical,
            "encode_host_GBps": round(wl5.raw_bytes / wl5.encode_s / 1e9, 2),
            "encode": f"the columns encoded on the GPU from values in HBM (adaptive cascade at ratio 2.0, "
                      f"Basic LZ4 / None; pa_amd.encode_table_device: one C-ABI call per column, four columns in "
                      f"flight on four contexts / streams); compared byte for byte with "
                      f"the host C++ writer's chunks ({threads} host threads, encode_host_GBps); the decode "
                      f"steps read the device-encoded chunks",
            "raw_bytes_this_rank": wl5.raw_bytes,
            "bit_exact": bool(ok5),
            "scaling": "strong",
            "parallelism": f"columns round-robin over {world} rank(s) (column ci on rank ci % {world})",
            "decode_units": f"{wl5.n_launch_units} plans per step: fixed-width / Boolean leaves grouped by type and "
                            f"nullability (pa_amd.ColumnGroupDecoder), one per Utf8 leaf; longest first over 4 streams",
            "traffic": load_traffic("c5_mixed_64col"),
        }
        if do_cpu:
            extra["c5_mixed_64col"]["cpu_baseline"] = wl5.cpu_baseline()
        del wl5

    if not args.no_encode:
        extra["encode_gpu"] = encode_gpu(torch, pa_amd, args.encode_rows, local, threads, args.steps)

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
                "workload": "c2_int32_adaptive_bitpack_dict",
                "rows": world * args.rows,
                "rows_this_rank": wl.rows,
                "page_rows": PAGE_ROWS,
                "pages_this_rank": len(wl.metas),
                "codec_mix": wl.mix,
                "compress_ratio_option": 1.2,
                "compressed_bytes_this_rank": wl.in_bytes,
                "decoded_bytes_this_rank": wl.out_bytes,
                "parallelism": f"page-shard x{world}: one column of {world} x {args.rows} rows cut by shard_pages, "
                               f"each rank decodes its range (for_shard), no collective on the data path",
            },
            "bit_exact": (not any_bad),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": load_traffic("c2_int32_adaptive_bitpack_dict"),
                "kernel": "k_decode_staged<4,false>",
                "kernel_ms": round(kavg, 4),
                "kernel_clock": "HIP events on the launch stream before the first and after the last timed step, span / steps",
                "frac_wall": round((wl.in_bytes + wl.out_bytes) / (wall_max / args.steps) / 1e9 / HBM_PEAK_GBPS, 4),
                "bytes_per_launch": wl.in_bytes + wl.out_bytes,
            },
        }
        line.update(extra)
        if do_cpu:
            line["cpu_baseline"] = cpu_baseline(wl)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
