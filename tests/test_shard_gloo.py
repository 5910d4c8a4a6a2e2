"""N>1 path on CPU: world_size 2 over gloo.  Each rank takes its page range
of one column chunk (pa_amd.shard_pages), decodes it (the
oracle stands in for the GPU here), and the shards gathered in rank order
equal the whole-column decode; the bench's max-over-ranks timing reduction
is exercised the same way."""
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


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import pa_amd
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    v = rng.integers(0, 1 << 14, 50000).astype(np.int32)
    chunk, metas = pa_amd.encode_column(v, None, False, pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=4096))
    shards = pa_amd.shard_pages(metas, world)
    me = shards[rank]
    mine = chunk[me.byte_offset:me.byte_offset + me.byte_len]
    out, _ = O.read_column(mine, [(m.length, m.num_values) for m in metas[me.page_begin:me.page_end]], np.int32)
    assert len(out) == me.rows
    sizes = [s.rows for s in shards]
    buf = torch.zeros(max(sizes), dtype=torch.int32)
    buf[: me.rows] = torch.from_numpy(out)
    gathered = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(gathered, buf)
    full = np.concatenate([g[:n].numpy() for g, n in zip(gathered, sizes)])
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, bool((full == v).all()), float(t[0])))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_page_shards_reassemble(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert all(t == float(world) for _, _, t in res)


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
