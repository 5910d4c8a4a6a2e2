"""bench.py's N>1 partitioning on the CPU (world size 2 over gloo): every
rank builds its provisional blocks of ONE column, the ranks all-gather the
page metas, pa_amd.shard_pages cuts the column, and each rank keeps its
range (bench.ShardedColumn).  The ranks' shards must tile the column that a
single rank builds alone -- same page bytes, same metas, same values, in
order, with no page twice -- and the C4 List shards likewise."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROWS = 9 * 8192 * 64 // 8 + 4321  # 1.5 blocks of pages per rank at world 2, a short last page


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_block(pa, seed):
    import bench

    def mk(b, r0, n):
        v = bench.gen_c2(n, seed, "mix", r0)
        opts = pa.WriteOptions(default_compress_ratio=1.2, max_page_size=bench.PAGE_ROWS, seed=seed * 1000003 + b)
        chunk, metas = pa.encode_column(v, None, False, opts, n_threads=2)
        return v, chunk, metas

    return mk


def _worker(rank, world, port, q):
    import torch.distributed as dist

    import bench
    import pa_amd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    col = bench.ShardedColumn(pa_amd, dist, world, rank, ROWS, _make_block(pa_amd, 42))
    vals = col.flat_values()
    parts = [None] * world
    dist.all_gather_object(parts, (col.global_shard, col.chunk, [(m.length, m.num_values) for m in col.metas],
                                   vals.tobytes(), col.shard.row_offset, col.rows))
    q.put((rank, parts))
    dist.destroy_process_group()


def test_sharded_column_tiles_the_column():
    import bench
    import pa_amd

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts = res[0][1]
    whole = bench.ShardedColumn(pa_amd, None, 1, 0, ROWS, _make_block(pa_amd, 42))
    assert b"".join(p[1] for p in parts) == whole.chunk
    assert sum((p[2] for p in parts), []) == [(m.length, m.num_values) for m in whole.metas]
    assert b"".join(p[3] for p in parts) == whole.flat_values().tobytes()
    assert np.array_equal(whole.flat_values(), bench.gen_c2(ROWS, 42, "mix"))
    assert [p[4] for p in parts] == [0, parts[0][5]] and parts[0][5] + parts[1][5] == ROWS
    g0, g1 = parts[0][0], parts[1][0]
    assert g0.page_end == g1.page_begin and g1.page_end == len(whole.metas)
    assert abs(g0.byte_len - g1.byte_len) <= max(m.length for m in whole.metas)
