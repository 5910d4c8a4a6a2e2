"""N>1 path on CPU: world_size 2 over gloo.  Each rank
takes its page range of a column chunk (pa_amd.shard_pages), decodes it --
with pa_amd's decoders (ColumnDecoder / BinaryColumnDecoder /
ListColumnDecoder .for_shard) when a GPU is present, else with the oracle
standing in -- and places it in the whole column: flat rows at the shard's
row_offset; Utf8 offsets rebased by the exclusive scan of the ranks' value
bytes, List offsets by the scan of their leaf counts (pa_amd.gather_sizes /
exclusive_bases, one all-gather).  The reassembled column must equal the
whole-column decode of the oracle bit for bit; the bench's max-over-ranks
timing reduction is exercised the same way."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _columns():
    import pa_amd

    rng = np.random.default_rng(5)
    v = rng.integers(0, 1 << 14, 50000).astype(np.int32)
    opts = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=4096)
    ichunk, imetas = pa_amd.encode_column(v, None, False, opts)
    strs = [str(x).encode() * int(rng.integers(0, 3)) for x in rng.integers(0, 10**6, 30000)]
    svals, soffs = pa_amd.binary.strings_to_arrow(strs)
    svalid = rng.random(len(strs)) > 0.1
    schunk, smetas = pa_amd.encode_binary_column(svals, soffs, svalid, True,
                                                 pa_amd.WriteOptions(default_compression=1, max_page_size=2048))
    lens = rng.integers(0, 6, 20000)
    loffs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    child = rng.integers(-1000, 1000, int(loffs[-1])).astype(np.int64)
    lchunk, lmetas = pa_amd.encode_list_column(loffs, child, None, None, False, False,
                                               pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=1500))
    return (ichunk, imetas), (schunk, smetas), (lchunk, lmetas)


def _decode(kind, chunk, metas, sh, gpu):
    """(offsets|None, values, validity|None) of one shard, as numpy."""
    import pa_amd
    from oracle import oracle as O

    if gpu:
        import torch

        d = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda()
        if kind == "int":
            dec = pa_amd.ColumnDecoder.for_shard(d, metas, sh, np.int32, False)
            v, _ = dec.decode()
            return None, v.cpu().numpy()[:dec.num_rows], None
        if kind == "utf8":
            dec = pa_amd.BinaryColumnDecoder.for_shard(d, metas, sh, pa_amd.UTF8, True)
            o, v, m = dec.decode()
            valid = pa_amd.read.unpack_bitmap(m, dec.num_rows).cpu().numpy()
            return o.cpu().numpy().astype(np.int64), v[:dec.values_bytes].cpu().numpy().tobytes(), valid
        dec = pa_amd.ListColumnDecoder.for_shard(d, metas, sh, np.int64, False, False)
        o, _, v, _ = dec.decode()
        return o.cpu().numpy().astype(np.int64), v.cpu().numpy()[:dec.num_leaves], None
    part, pm = pa_amd.shard_slice(chunk, metas, sh)
    pm = [(m.length, m.num_values) for m in pm]
    if kind == "int":
        v, _ = O.read_column(part, pm, np.int32)
        return None, v, None
    if kind == "utf8":
        return O.read_binary_column(part, pm, True)
    o, _, v, _ = O.read_list_column(part, pm, np.int64, False, False)
    return o, v, None


def _worker(rank, world, port, q, need_gpu=False):
    import torch
    import torch.distributed as dist

    import pa_amd
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gpu = torch.cuda.is_available()
    if need_gpu and not gpu:
        q.put((rank, {"gpu": False}, 0.0))
        return
    ok = {}
    for kind, (chunk, metas) in zip(("int", "utf8", "list"), _columns()):
        shards = pa_amd.shard_pages(metas, world)
        me = shards[rank]
        offs, vals, valid = _decode(kind, chunk, metas, me, gpu)
        whole = [(m.length, m.num_values) for m in metas]
        parts = [None] * world
        if kind == "int":
            assert len(vals) == me.rows
            dist.all_gather_object(parts, (me.row_offset, vals))
            full = np.concatenate([p[1] for p in sorted(parts, key=lambda p: p[0])])
            ok[kind] = bool((full == O.read_column(chunk, whole, np.int32)[0]).all())
            continue
        # variable-size outputs: this rank's base from the scan of all ranks' sizes
        nvals = len(vals)
        base = pa_amd.shard_base(nvals, rank)
        rows_base = pa_amd.shard_base(len(offs) - 1, rank)
        g = pa_amd.rebase_offsets(offs, base)
        dist.all_gather_object(parts, (rows_base, g, vals, valid))
        parts.sort(key=lambda p: p[0])
        go = np.concatenate([parts[0][1][:1]] + [p[1][1:] for p in parts])
        if kind == "utf8":
            eo, ev, em = O.read_binary_column(chunk, whole, True)
            gv = b"".join(p[2] for p in parts)
            gm = np.concatenate([p[3] for p in parts])
            ok[kind] = bool((go == eo).all() and gv == ev and (gm == em).all())
        else:
            eo, _, ev, _ = O.read_list_column(chunk, whole, np.int64, False, False)
            gv = np.concatenate([p[2] for p in parts])
            ok[kind] = bool((go == eo).all() and (gv == ev).all())
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, ok, float(t[0])))
    dist.destroy_process_group()


def _run(world, need_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, need_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, ok, _ in res:
        assert ok == {"int": True, "utf8": True, "list": True}, ok
    assert all(t == float(world) for _, _, t in res)


@pytest.mark.parametrize("world", [2])
def test_page_shards_reassemble(world):
    _run(world, False)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2])
def test_page_shards_reassemble_gpu(world):
    """The same under a real process group with both ranks on the box's GPU:
    every rank plans and decodes its page range with pa_amd's HIP decoders
    (for_shard), the bases come from the all-gather, and the reassembled
    columns match the oracle's whole-column decode."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run(world, True)


def test_exclusive_bases():
    import pa_amd

    assert pa_amd.exclusive_bases([3, 0, 5, 2]) == [0, 3, 3, 8]


def test_shard_pages_balanced():
    import pa_amd

    metas = [pa_amd.PageMeta(1000 + 10 * (i % 7), 8192) for i in range(1000)]
    for world in (1, 2, 4, 8):
        sh = pa_amd.shard_pages(metas, world)
        assert sh[0].page_begin == 0 and sh[-1].page_end == len(metas)
        assert all(a.page_end == b.page_begin for a, b in zip(sh, sh[1:]))
        lens = [s.byte_len for s in sh]
        assert max(lens) - min(lens) <= 2 * 1070
        assert sum(s.rows for s in sh) == 8192 * 1000


# ---- world size 4: bench.py's own partitioning, oracle standing in ----------
def _bench_worker(rank, world, port, q):
    """One rank of bench.py's N>1 legs on CPU: the C4-shaped List<Int32>
    column and the C2 column through bench.ShardedColumn (provisional blocks,
    all-gathered page metas, shard_pages), C5's columns round-robin
    (WorkloadC5.rank_columns); each rank decodes its part with the oracle and
    the parts are reassembled on rank 0 against whole-column decodes."""
    import torch.distributed as dist

    import bench
    import pa_amd
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = 3 * bench.BLOCK_PAGES * 512  # per rank; blocks of 64 pages of PAGE_ROWS rows are too big for CPU
    out = {}
    saved = bench.PAGE_ROWS
    bench.PAGE_ROWS = 512
    try:
        def c2_block(b, r0, n):
            v = bench.gen_c2(n, 7, "mix", r0)
            opts = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=bench.PAGE_ROWS, seed=7 + b)
            chunk, metas = pa_amd.encode_column(v, None, False, opts)
            return v, chunk, metas

        col = bench.ShardedColumn(pa_amd, dist, world, rank, world * rows, c2_block)
        vals, _ = O.read_column(col.chunk, [(m.length, m.num_values) for m in col.metas], np.int32)
        parts = [None] * world
        dist.all_gather_object(parts, (col.global_shard.row_offset, vals, col.flat_values()))
        if rank == 0:
            parts.sort(key=lambda p: p[0])
            full = np.concatenate([p[1] for p in parts])
            src = np.concatenate([p[2] for p in parts])
            out["c2"] = bool(len(full) == world * rows and (full == src).all()
                             and (full == bench.gen_c2(world * rows, 7, "mix")).all())

        def l_block(b, r0, n):
            rng = np.random.default_rng([99, b])
            ln = rng.integers(0, 3, n)
            lv = rng.random(n) >= 0.1
            ln[~lv] = 0
            offs = np.zeros(n + 1, np.int64)
            np.cumsum(ln, out=offs[1:])
            child = rng.integers(0, 1 << 16, int(offs[-1])).astype(np.int32)
            cv = rng.random(len(child)) >= 0.2
            opts = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=bench.PAGE_ROWS, seed=b)
            chunk, metas = pa_amd.encode_list_column(offs, child, lv, cv, True, True, opts)
            return (offs, child, lv, cv), chunk, metas

        col = bench.ShardedColumn(pa_amd, dist, world, rank, world * rows, l_block)
        m = [(x.length, x.num_values) for x in col.metas]
        offs, lv, child, cv = O.read_list_column(col.chunk, m, np.int32, True, True)
        leaf_base = pa_amd.shard_base(len(child), rank)  # the one exchange (setup only)
        parts = [None] * world
        dist.all_gather_object(parts, (col.global_shard.row_offset, offs + leaf_base, lv, child, cv))
        if rank == 0:
            parts.sort(key=lambda p: p[0])
            go = np.concatenate([parts[0][1][:1]] + [p[1][1:] for p in parts])
            nb = (world * rows + bench.BLOCK_PAGES * bench.PAGE_ROWS - 1) // (bench.BLOCK_PAGES * bench.PAGE_ROWS)
            whole, wm = b"", []
            for b in range(nb):
                r0 = b * bench.BLOCK_PAGES * bench.PAGE_ROWS
                _, ch, mt = l_block(b, r0, min(bench.BLOCK_PAGES * bench.PAGE_ROWS, world * rows - r0))
                whole += ch
                wm += [(x.length, x.num_values) for x in mt]
            eo, elv, ec, ecv = O.read_list_column(whole, wm, np.int32, True, True)
            out["c4"] = bool((go == eo).all() and (np.concatenate([p[2] for p in parts]) == elv).all()
                             and (np.concatenate([p[3] for p in parts]) == ec).all()
                             and (np.concatenate([p[4] for p in parts]) == ecv).all())

        specs = bench.WorkloadC5.specs()
        mine = bench.WorkloadC5.rank_columns(len(specs), world, rank)
        n5 = 3000
        got = {}
        for ci in mine:
            dt, kind = specs[ci]
            v, valid, nullable, _, chunk, metas, _ = bench.WorkloadC5.host_column(pa_amd, dt, kind, ci, n5, 555, 1)
            m = [(x.length, x.num_values) for x in metas]
            if dt == "utf8":
                o, b, _ = O.read_binary_column(chunk, m, False)
                ok = b == v[0] and (o == v[1]).all()
            elif dt == np.bool_:
                bits, vv = O.read_bool_column(chunk, m, nullable)
                keep = valid if nullable else np.ones(n5, bool)
                ok = (bits[keep] == v[keep]).all() and (not nullable or (vv == valid).all())
            else:
                x, vv = O.read_column(chunk, m, dt, nullable)
                keep = valid if nullable else np.ones(n5, bool)
                ok = (x[keep] == v[keep]).all() and (not nullable or (vv == valid).all())
            got[ci] = bool(ok)
        parts = [None] * world
        dist.all_gather_object(parts, got)
        if rank == 0:
            allc = {}
            for d in parts:
                assert not set(d) & set(allc), "a column decoded on two ranks"
                allc.update(d)
            out["c5"] = sorted(allc) == list(range(len(specs))) and all(allc.values())
    finally:
        bench.PAGE_ROWS = saved
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_bench_partitions_world(world):
    """bench.py's C2 / C4 page shards and C5 column round-robin at world
    size 4 and 8 over gloo (the 4-GPU C4 and 8-GPU C5 splits rehearsed on
    CPU): the reassembled columns equal the whole-column oracle decodes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == {"c2": True, "c4": True, "c5": True}, res[0]
