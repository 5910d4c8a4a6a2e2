"""Page sharding across the GPUs of a node.

Pages are self-describing given PageMeta.num_values (src/lib.rs:75-80) and
no decoder carries state across pages (delta chains and Patas restart per
page: delta_bp.rs:73, patas.rs:108-117), so a column chunk splits into
contiguous page ranges, one per rank, balanced by compressed bytes.  Fixed-
width outputs need no exchange: each rank's first output row is the running
sum of num_values, known from the footer on every rank.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence


@dataclass(frozen=True)
class Shard:
    rank: int
    page_begin: int
    page_end: int
    byte_offset: int  # into the column chunk
    byte_len: int
    row_offset: int
    rows: int


def shard_pages(metas: Sequence, world: int) -> List[Shard]:
    """Contiguous page ranges with near-equal compressed bytes."""
    lengths = [int(m.length) for m in metas]
    total = sum(lengths)
    shards, p = [], 0
    byte_off = row_off = 0
    for r in range(world):
        target = total * (r + 1) / world
        begin = p
        acc = byte_off
        while p < len(metas) and (r == world - 1 or acc + lengths[p] / 2 <= target):
            acc += lengths[p]
            p += 1
        blen = sum(lengths[begin:p])
        rows = sum(int(m.num_values) for m in metas[begin:p])
        shards.append(Shard(r, begin, p, byte_off, blen, row_off, rows))
        byte_off += blen
        row_off += rows
    return shards


def shard_slice(chunk, metas: Sequence, shard: Shard):
    """The shard's bytes of the column chunk (host bytes or a device tensor
    view) and its page metas: a rank reads nothing outside its range."""
    return chunk[shard.byte_offset:shard.byte_offset + shard.byte_len], list(metas[shard.page_begin:shard.page_end])


def exclusive_bases(sizes: Sequence[int]) -> List[int]:
    """Exclusive scan: where each shard's variable-size output (Utf8 value
    bytes, List leaves) starts in the whole column."""
    out, acc = [], 0
    for s in sizes:
        out.append(acc)
        acc += int(s)
    return out


def gather_sizes(local: int, group=None) -> List[int]:
    """All ranks' local sizes in rank order (one int64 all-gather; gloo on
    CPU, RCCL when the process group is nccl and the tensor is on a GPU)."""
    import torch
    import torch.distributed as dist

    dev = "cpu"
    if dist.get_backend(group) == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"
    t = torch.tensor([int(local)], dtype=torch.int64, device=dev)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return [int(p.item()) for p in parts]


def shard_base(local: int, rank: int, group=None) -> int:
    """This rank's base in the whole column's variable-size output."""
    return exclusive_bases(gather_sizes(local, group))[rank]


def rebase_offsets(offsets, base: int):
    """A shard's offsets (starting at 0) moved onto the whole column's values:
    rows [row_offset, row_offset + rows] of the column's offsets."""
    return offsets + base
