"""Synthetic column builders for the parity tests (seeded numpy generators
restating the reference's tests/it/io.rs:343-415 shapes), paged and encoded
with the oracle's restatement of NativeWriter::encode_chunk
(write/common.rs:49-119: fixed-row pages, last page shorter)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


def gen_values(kind: str, n: int, dtype, rng: np.random.Generator, uniq: int = 1000) -> np.ndarray:
    dt = np.dtype(dtype)
    info = np.iinfo(dt) if dt.kind in "iu" else None
    if kind == "index":  # create_random_index: ints in [0, uniq)
        v = rng.integers(0, uniq, n)
    elif kind == "full":  # the type's whole range
        if dt.kind == "f":
            return rng.standard_normal(n).astype(dt) * 1e4
        v = rng.integers(info.min, info.max, n, endpoint=True, dtype=np.int64 if dt.itemsize < 8 or dt.kind == "i" else np.uint64)
    elif kind == "sorted":
        v = np.sort(rng.integers(0, uniq * 100 + 1, n))
    elif kind == "one":
        v = np.full(n, 7)
    elif kind == "runs":
        v = np.repeat(rng.integers(0, 50000, n // 37 + 2), 37)[:n]
    elif kind == "short_runs":
        lens = rng.choice([2, 3], size=n // 2 + 1, p=[0.3, 0.7])
        v = np.repeat(rng.integers(0, 2**31 - 1, len(lens)), lens)[:n]
    elif kind == "freq":
        v = np.where(rng.random(n) < 0.95, 300, rng.integers(0, 10000, n))
    elif kind.startswith("bits"):  # uniform in [0, 2^b)
        b = int(kind[4:])
        v = rng.integers(0, 2**b, n, dtype=np.uint64)
    else:
        raise ValueError(kind)
    if dt.kind == "f":
        return np.asarray(v).astype(dt)
    if info is not None:
        v = np.asarray(v)
        if v.dtype.kind == "f":
            v = v.astype(np.int64)
        v = v.astype(np.uint64) & np.uint64((1 << (8 * dt.itemsize)) - 1) if dt.itemsize < 8 else v
    return np.asarray(v).astype(dt)


def build_column(values: np.ndarray, validity, nullable: bool, page_rows: int, opts: O.WriteOptions):
    """-> (chunk bytes, [(length, num_values)], codecs per page)."""
    n = len(values)
    pages, metas, codecs = [], [], []
    step = page_rows if page_rows else max(n, 1)
    for off in range(0, n, step):
        m = min(step, n - off)
        v = values[off:off + m]
        val = None if validity is None else validity[off:off + m]
        pg = O.write_page(v, val, nullable, opts)
        pages.append(pg)
        metas.append((len(pg), m))
        codecs.append(O.page_codec(pg, nullable))
    return b"".join(pages), metas, codecs


def oracle_decode_column(chunk: bytes, metas, dtype, nullable: bool):
    """Oracle read of every page, appended (read_integer / read_double)."""
    vals, valid = [], []
    pos = 0
    for length, nv in metas:
        v, m = O.read_page(chunk[pos:pos + length], nv, dtype, nullable)
        vals.append(v)
        if nullable:
            valid.append(m)
        pos += length
    values = np.concatenate(vals) if vals else np.zeros(0, dtype)
    validity = np.concatenate(valid) if nullable and valid else (np.zeros(0, bool) if nullable else None)
    return values, validity


def page_codecs(chunk: bytes, metas, nullable: bool) -> list:
    """The codec byte of every page of a chunk ([(length, num_values)])."""
    out, pos = [], 0
    for length, _ in metas:
        out.append(O.page_codec(chunk[pos:pos + length], nullable))
        pos += length
    return out


def same_pages_but_zstd(dev: bytes, dev_metas, host: bytes, host_metas, nullable: bool) -> list:
    """A Zstd-default chunk from the device encoder against the host writer's:
    the device's frames come from sb_zstdc.h, not libzstd level 3, so the bar
    is decode equivalence -- the same pages (row counts) with the same codec
    choices.  Returns the device's (length, num_values) metas."""
    dm = [(m.length, m.num_values) for m in dev_metas]
    hm = [(m.length, m.num_values) for m in host_metas]
    assert [nv for _, nv in dm] == [nv for _, nv in hm]
    assert sum(length for length, _ in dm) == len(dev)
    assert page_codecs(dev, dm, nullable) == page_codecs(host, hm, nullable)
    return dm
