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
