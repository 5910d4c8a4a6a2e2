"""Writer-legal fixed-width pages larger than one workgroup's LDS (SURVEY
§8 a7 / a8): the reference's default `max_page_size = None` writes one page
per column chunk (write/common.rs:54-58), so Dict / Freq cascades over
millions of rows are ordinary output.

* Freq pages with more roaring containers than the LDS tables hold
  (integer/freq.rs:88-123): the container tables are built by the workgroup
  into the page's HBM region -- 1M rows (16 bitmap containers), 3M rows
  (46 containers);
* Dict / Freq cascades whose general-codec (LZ4 / Zstd / Snappy) or Patas
  leaf expands past the deferred pass's LDS: the leaf is expanded into the
  page's region by k_inflate / k_zinflate and the page decoded from there
  (k_decode_spilled) -- a 1M-row Dict page with an LZ4 index stream, an Int64
  forced-Freq page of 8192 / 16384 incompressible exceptions under Zstd, a
  Float64 Freq page whose exceptions are Patas.

Each decode is compared bit for bit (values under nulls included) with the
oracle's read_column."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


def check(pa_amd, ctx, v, valid, nullable, page_rows=0, **kw):
    chunk, metas = pa_amd.encode_column(v, valid, nullable, pa_amd.WriteOptions(max_page_size=page_rows, **kw))
    dt = v.dtype
    dec = pa_amd.ColumnDecoder(chunk, metas, dt, nullable, ctx)
    for _ in range(2):  # both work-list parities
        got, gm = dec.decode()
    ev, em = O.read_column(chunk, [(m.length, m.num_values) for m in metas], dt, nullable)
    g = got.cpu().numpy().view(np.uint8)[: ev.nbytes].view(dt)
    gb, eb = g.view(np.uint8).reshape(-1, dt.itemsize), ev.view(np.uint8).reshape(-1, dt.itemsize)
    bad = np.flatnonzero((gb != eb).any(1))
    assert len(bad) == 0, f"{len(bad)} rows differ, first at {bad[:5]}: {g[bad[:5]]} vs {ev[bad[:5]]}"
    if nullable:
        assert (pa_amd.read.unpack_bitmap(gm, len(v)).cpu().numpy() == em).all(), "validity differs"
    return chunk, metas


def codec_of(chunk, nullable):
    q = 4 + int.from_bytes(chunk[:4], "little") if nullable else 0
    return chunk[q]


@pytest.mark.parametrize("rows,top", [(1 << 20, 0.91), (1 << 20, 0.96), (3_000_000, 0.91), (70_000, 0.92)])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_freq_many_containers(ctx, rows, top, nullable):
    """One Freq page over `rows` rows: 1M rows at 9 % exceptions = 16 bitmap
    containers, at 4 % = 16 array containers; 3M rows = 46 containers."""
    import pa_amd

    rng = np.random.default_rng(rows)
    v = np.where(rng.random(rows) < top, 300, rng.integers(0, 1 << 20, rows)).astype(np.int32)
    valid = rng.random(rows) > 0.05 if nullable else None
    chunk, _ = check(pa_amd, ctx, v, valid, nullable, default_compress_ratio=1.2)
    assert codec_of(chunk, nullable) == 13


@pytest.mark.parametrize("codec", [1, 2, 3], ids=["lz4", "zstd", "snappy"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_dict_general_index_stream_1m(ctx, codec, nullable):
    """A 1M-row Dict page whose index stream is the default general codec
    (forced Dict, ratio None: the nested call may not use Dict again and
    falls back to the default codec): 4 MiB of indices spill to HBM."""
    import pa_amd

    rng = np.random.default_rng(7 + codec)
    rows = 1 << 20
    v = rng.integers(0, 2**31, 1000)[rng.integers(0, 1000, rows)].astype(np.int32)
    valid = rng.random(rows) > 0.1 if nullable else None
    chunk, _ = check(pa_amd, ctx, v, valid, nullable, default_compression=codec, forced_codec=11)
    assert codec_of(chunk, nullable) == 11


@pytest.mark.parametrize("rows", [8192, 16384, 200_000])
def test_int64_forced_freq_zstd_incompressible(ctx, rows):
    """Forced Freq over incompressible Int64 under Zstd: rows - 1 exceptions
    in a Zstd frame whose expansion plus the page exceed the LDS."""
    import pa_amd

    rng = np.random.default_rng(rows)
    v = rng.integers(-2**62, 2**62, rows).astype(np.int64)
    v[rows // 3] = v[0]  # one repeat: the top value
    chunk, _ = check(pa_amd, ctx, v, None, False, default_compression=2, forced_codec=13)
    assert codec_of(chunk, False) == 13


@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
def test_float64_freq_patas_exceptions(ctx, nullable):
    """A 1M-row Float64 Freq page whose exceptions stream is Patas (a slowly
    varying walk): 800 KiB of exceptions expand in HBM (k_inflate Patas)."""
    import pa_amd

    rng = np.random.default_rng(11)
    rows = 1 << 20
    walk = 1000.0 + np.cumsum(rng.integers(1, 64, rows)) * 2.0**-20
    v = np.where(rng.random(rows) < 0.91, 0.5, walk)
    valid = rng.random(rows) > 0.1 if nullable else None
    chunk, _ = check(pa_amd, ctx, v, valid, nullable, default_compress_ratio=1.2, forced_codec=13)
    assert codec_of(chunk, nullable) == 13


@pytest.mark.parametrize("codec", [1, 2], ids=["lz4", "zstd"])
def test_spill_pages_beside_small_pages(ctx, codec):
    """Small and large pages in one column: only the large one spills, the
    work lists of both decode parities stay consistent."""
    import pa_amd

    rng = np.random.default_rng(99)
    parts = []
    for rows in (8192, 1 << 20, 5000, 300_000):
        parts.append(rng.integers(0, 2**31, 500)[rng.integers(0, 500, rows)].astype(np.int32))
    chunks, metas = [], []
    for p in parts:
        c, m = pa_amd.encode_column(p, None, False, pa_amd.WriteOptions(max_page_size=0, default_compression=codec,
                                                                          forced_codec=11))
        chunks.append(c)
        metas += m
    chunk = b"".join(chunks)
    v = np.concatenate(parts)
    dec = pa_amd.ColumnDecoder(chunk, metas, np.int32, False, ctx)
    for _ in range(3):
        got, _ = dec.decode()
        assert np.array_equal(got.cpu().numpy()[: len(v)], v)
