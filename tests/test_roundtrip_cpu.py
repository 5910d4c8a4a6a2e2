"""The reference's integration matrix (tests/it/io.rs:72-278 via
test_write_read :417-438) restated for flat primitive columns: every chunk is
written under None / LZ4 / Zstd / Snappy with 2048-row pages and
default_compress_ratio 2.0, read back, and compared with Arrow logical
equality (values under null slots are not compared, like assert_eq!).
Writer = the product's host encoder; reader = the oracle (CPU).  The GPU
reader is held to the same pages, bit-exact, in test_gpu_*.py."""
import numpy as np
import pytest

import pa_amd
from oracle import oracle as O

WRITE_PAGE = 2048
CODECS = [0, 1, 2, 3]


def write_read(values, validity, nullable):
    for dc in CODECS:
        opts = pa_amd.WriteOptions(default_compression=dc, default_compress_ratio=2.0, max_page_size=WRITE_PAGE,
                                   forbidden_compressions=(O.PATAS,) if values.dtype == np.float32 else ())
        chunk, metas = pa_amd.encode_column(values, validity, nullable, opts)
        assert sum(m.num_values for m in metas) == len(values)
        out, vv = O.read_column(chunk, [(m.length, m.num_values) for m in metas], values.dtype, nullable)
        if nullable:
            assert (vv == validity).all()
            m = validity
            assert (out[m].view(np.uint8) if out.dtype.itemsize == 1 else out[m]).tobytes() == values[m].tobytes()
        else:
            assert out.tobytes() == values.tobytes()


def create_random_index(size, null_density, uniq, rng, dtype=np.int32):
    v = rng.integers(0, uniq, size).astype(dtype)
    valid = rng.random(size) >= null_density
    return v, valid


def test_basic():
    for dt in [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16, np.int32, np.int64, np.float32, np.float64]:
        v = np.array([1, 2, 3, 4, 5, 6], dtype=dt) if np.dtype(dt).kind != "f" else np.array([1.1, 2.2, 3.3, 4.4, 5.5, 6.6], dt)
        write_read(v, None, False)


@pytest.mark.parametrize("null_density", [0.0, 0.1, 0.2, 0.3, 0.4, 0.5])
def test_random(null_density):
    rng = np.random.default_rng(42)
    for dt in [np.int32, np.int64, np.float64]:
        v, valid = create_random_index(10000, null_density, 10000, rng, dt)
        write_read(v, valid, True)
        write_read(v, None, False)


def test_dict():
    rng = np.random.default_rng(42)
    for nd in [0.1, 0.2, 0.3, 0.4]:
        v, valid = create_random_index(10000, nd, 8, rng)
        write_read(v, valid, True)
    v, valid = create_random_index(10000, 0.5, 8, rng, np.float64)
    write_read(v, valid, True)


def test_freq():
    # io.rs:120-132: per page 2045 x 20 + 3 x 10000
    page = np.concatenate([np.full(2045, 20, np.uint32), np.full(3, 10000, np.uint32)])
    v = np.tile(page, 5)
    write_read(v, None, False)
    opts = pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=WRITE_PAGE)
    chunk, metas = pa_amd.encode_column(v, None, False, opts)
    assert chunk[0] == O.FREQ


def test_bitpacking():
    rng = np.random.default_rng(42)
    v, _ = create_random_index(10240, 0.0, 8, rng)
    write_read(v, None, False)


def test_delta_bitpacking():
    # io.rs:146-152: 0..10240 as u32 and i32
    for dt in (np.uint32, np.int32):
        v = np.arange(10240, dtype=dt)
        write_read(v, None, False)
        chunk, metas = pa_amd.encode_column(v, None, False, pa_amd.WriteOptions(default_compress_ratio=2.0, max_page_size=WRITE_PAGE))
        assert chunk[0] == O.DELTA_BITPACKING


def test_onevalue():
    write_read(np.full(10000, 3, np.int32), None, False)
    write_read(np.full(10000, 3.5, np.float64), None, False)


def test_float():
    rng = np.random.default_rng(42)
    for nd in [0.0, 0.1, 0.5]:
        v = rng.integers(0, 10000, 10000).astype(np.float64)
        write_read(v, rng.random(10000) >= nd, True)
        v32 = np.round(rng.standard_normal(10000), 3).astype(np.float32)
        write_read(v32, None, False)


def test_encoder_matches_oracle_encoder():
    """Product host encoder == oracle restatement of compress_integer /
    compress_double, byte for byte, per page (same sampler seed)."""
    from tests.colgen import gen_values

    rng = np.random.default_rng(1)
    for dt in [np.int32, np.uint32, np.int64, np.uint8, np.int16, np.float64]:
        for kind in ["index", "full", "sorted", "one", "runs", "short_runs", "freq", "bits12"]:
            v = gen_values(kind, 9000, dt, rng)
            for nullable in (False, True):
                val = rng.random(9000) > 0.2 if nullable else None
                for ratio, forced, dc in [(None, -1, 0), (1.2, -1, 0), (2.0, O.DICT, 0), (2.0, O.FREQ, 0), (1.1, -1, 1)]:
                    wo = pa_amd.WriteOptions(default_compression=dc, default_compress_ratio=ratio, max_page_size=4096,
                                             forced_codec=forced, seed=11)
                    chunk, metas = pa_amd.encode_column(v, val, nullable, wo)
                    pos = 0
                    for i, m in enumerate(metas):
                        sl = slice(i * 4096, i * 4096 + m.num_values)
                        ob = O.write_page(v[sl], None if val is None else val[sl], nullable,
                                          O.WriteOptions.make(default_codec=dc, ratio=ratio, forced=forced,
                                                              seed=pa_amd.page_seed(11, i)))
                        assert chunk[pos:pos + m.length] == ob, (np.dtype(dt).name, kind, nullable, ratio, forced, i)
                        pos += m.length


@pytest.mark.parametrize("P", [70_000, 300_000])
def test_encoder_matches_oracle_encoder_big_pages(P):
    """Pages past 65 535 rows: the product writer's 64-bit statistics table
    words and multi-container roaring bitmaps (roaring 0.10.1 serialize_into)
    against the oracle restatement, byte for byte.  The device encoder is
    pinned to the product writer at these sizes (test_gpu_encode.py), so
    this closes the chain to the restatement."""
    from tests.colgen import gen_values

    rng = np.random.default_rng(P)
    n = P + P // 3  # a full page and a short one
    cases = [(np.int32, "freq"), (np.int64, "freq"), (np.int32, "index"), (np.float64, "freq"), (np.uint32, "runs"),
             (np.int32, "sorted"), (np.float64, "index")]
    for dt, kind in cases:
        v = gen_values(kind, n, dt, rng)
        for nullable in (False, True):
            val = rng.random(n) > 0.1 if nullable else None
            for ratio, forced in [(1.2, -1), (2.0, O.FREQ), (2.0, O.DICT)]:
                wo = pa_amd.WriteOptions(default_compress_ratio=ratio, max_page_size=P, forced_codec=forced, seed=5)
                chunk, metas = pa_amd.encode_column(v, val, nullable, wo)
                pos = 0
                for i, m in enumerate(metas):
                    sl = slice(i * P, i * P + m.num_values)
                    ob = O.write_page(v[sl], None if val is None else val[sl], nullable,
                                      O.WriteOptions.make(ratio=ratio, forced=forced, seed=pa_amd.page_seed(5, i)))
                    assert chunk[pos:pos + m.length] == ob, (np.dtype(dt).name, kind, nullable, ratio, forced, i)
                    pos += m.length


def test_binary_encoder_matches_oracle_encoder_big_pages():
    """Utf8 pages past 65 535 rows (Freq with several roaring containers,
    Dict, adaptive) against the oracle's binary writer."""
    rng = np.random.default_rng(9)
    P = 140_000
    n = P + 1000
    pool = [f"v{i}".encode() for i in range(300)]
    strs = [b"common" if r < 0.93 else pool[i] for r, i in zip(rng.random(n), rng.integers(0, 300, n))]
    vals, offs = pa_amd.binary.strings_to_arrow(strs)
    valid = rng.random(n) > 0.1
    for ratio, forced in [(2.0, O.FREQ), (2.0, O.DICT), (1.2, -1)]:
        wo = pa_amd.WriteOptions(default_compress_ratio=ratio, max_page_size=P, forced_codec=forced, seed=3)
        chunk, metas = pa_amd.encode_binary_column(vals, offs, valid, True, wo, physical_type=pa_amd.UTF8)
        pos = 0
        for i, m in enumerate(metas):
            r0, r1 = i * P, i * P + m.num_values
            po = offs[r0:r1 + 1] - offs[r0]
            ob = O.write_binary_page(vals[offs[r0]:offs[r1]], po, valid[r0:r1], True,
                                     O.WriteOptions.make(ratio=ratio, forced=forced, seed=pa_amd.page_seed(3, i)),
                                     parent_values_len=len(vals))
            assert chunk[pos:pos + m.length] == ob, (ratio, forced, i)
            pos += m.length


def _null_slot_column(n, dt, rng):
    """Valid rows small (< 2^8, or a slowly varying double), null slots
    holding 2^30-scale garbage: the sampled ratio of compress_sample_ratio
    must see T::default() there (integer/mod.rs:334-336 rebuilds the sample
    through MutablePrimitiveArray::extend_trusted_len, which writes zeros
    under None), not the slot's bits."""
    valid = rng.random(n) > 0.3
    if np.dtype(dt).kind == "f":
        v = np.round(np.cumsum(rng.integers(-1, 2, n)) * 0.25 + 100.0, 2).astype(dt)
        garbage = rng.standard_normal(n).astype(dt) * dt(1e300 if dt == np.float64 else 1e30)
    else:
        v = rng.integers(0, 256, n).astype(dt)
        garbage = rng.integers(2**30, 2**31, n).astype(dt)
    v = np.where(valid, v, garbage)
    return v, valid


def test_sample_ratio_null_slots_read_default():
    """The rule pinned: a nullable Int32 page whose null slots hold 2^30-scale
    values and whose valid rows are < 2^8 chooses Bitpacking (the sample's
    bit width comes from the zeros: b = 8, ratio ~3.97), not Dict (1.79, what
    a sample keeping the slots' bits, b = 31, ratio 1.03, leaves as the best).
    Oracle, host writer and the reference rule agree byte for byte."""
    rng = np.random.default_rng(77)
    n = 8192
    v, valid = _null_slot_column(n, np.int32, rng)
    page = O.write_page(v, valid, True, O.WriteOptions.make(ratio=1.2, seed=3))
    assert O.page_codec(page, True) == O.BITPACKING
    wo = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=n, seed=3)
    chunk, metas = pa_amd.encode_column(v, valid, True, wo)
    ob = O.write_page(v, valid, True, O.WriteOptions.make(ratio=1.2, seed=pa_amd.page_seed(3, 0)))
    assert chunk == ob
    out, vv = O.read_column(chunk, [(m.length, m.num_values) for m in metas], np.int32, True)
    assert out.tobytes() == v.tobytes() and (vv == valid).all()
    # every sampled candidate, for each type the writers sample: host == oracle
    for dt in (np.int32, np.uint32, np.int64, np.int16, np.float64, np.float32):
        v, valid = _null_slot_column(20000, dt, rng)
        for ratio, forbidden in ((1.2, ()), (1.0, (O.DICT, O.FREQ)), (2.0, (O.DICT,))):
            if dt == np.float32:
                forbidden = forbidden + (O.PATAS,)
            wo = pa_amd.WriteOptions(default_compress_ratio=ratio, max_page_size=4096, seed=9,
                                     forbidden_compressions=forbidden)
            chunk, metas = pa_amd.encode_column(v, valid, True, wo)
            pos = 0
            for i, m in enumerate(metas):
                sl = slice(i * 4096, i * 4096 + m.num_values)
                ob = O.write_page(v[sl], valid[sl], True, O.WriteOptions.make(
                    ratio=ratio, forbidden=forbidden, seed=pa_amd.page_seed(9, i)))
                assert chunk[pos:pos + m.length] == ob, (np.dtype(dt).name, ratio, i)
                pos += m.length
