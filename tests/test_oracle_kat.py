"""Known-answer tests that pin the oracle to published formats.

* Patas pack/unpack: the reference's own KAT (double/patas.rs:191-202).
* BitPacker4x (bitpacking 0.8.0, SIMD-BP128): layouts derived by hand from
  the 4-lane vertical design -- value 4*i+l at bit i*b of lane l, lane word k
  at byte 16*k + 4*l.  Not pinned by any reference test (round trips only,
  tests/it/io.rs:135-152): "parity unpinned" beyond these hand KATs.
* roaring 0.10.1 portable serialization (RoaringFormatSpec, cookie 12346).
* parquet2 encode_bool (hybrid RLE, bit width 1) for the def-level prefix
  (write/serialize.rs:200-215).
"""
import numpy as np
import pytest

from oracle import oracle as O


def test_patas_reference_kat():
    for p, (r, s, t) in [(692, (1, 2, 52)), (1026, (2, 8, 2))]:
        assert O.patas_pack(r, s, t) == p
        assert O.patas_unpack(p) == (r, s, t)
    # unpack quirk: zero significant bytes with tz < 63 reads as 8 (patas.rs:154-156)
    assert O.patas_unpack(O.patas_pack(3, 0, 10)) == (3, 8, 10)
    assert O.patas_unpack(O.patas_pack(3, 0, 63)) == (3, 0, 63)


def test_bp4x_b1_kat():
    v = np.zeros(128, np.uint32)
    v[[0, 1, 2, 3, 4, 127]] = 1
    assert O.bp4x_pack(v, 1) == bytes.fromhex("03000000010000000100000001000080")


def test_bp4x_b8_kat():
    v = np.arange(128, dtype=np.uint32)
    exp = bytearray(128)
    for i in range(32):
        for l in range(4):
            exp[16 * (i // 4) + 4 * l + (i % 4)] = 4 * i + l
    assert O.bp4x_pack(v, 8) == bytes(exp)


def test_bp4x_b16_kat():
    v = (np.arange(128, dtype=np.uint32) * 509) & 0xFFFF
    exp = bytearray(256)
    for i in range(32):
        for l in range(4):
            o = 16 * (i // 2) + 4 * l + 2 * (i % 2)
            exp[o:o + 2] = int(v[4 * i + l]).to_bytes(2, "little")
    assert O.bp4x_pack(v, 16) == bytes(exp)


def test_bp4x_b32_is_identity():
    v = np.random.default_rng(0).integers(0, 2**32, 128, dtype=np.uint64).astype(np.uint32)
    assert O.bp4x_pack(v, 32) == v.tobytes()


@pytest.mark.parametrize("b", range(33))
def test_bp4x_roundtrip_every_width(b):
    rng = np.random.default_rng(b)
    v = rng.integers(0, 2**b, 128, dtype=np.uint64).astype(np.uint32) if b else np.zeros(128, np.uint32)
    d = O.bp4x_pack(v, b)
    assert len(d) == 16 * b
    assert (O.bp4x_unpack(d, b) == v).all()
    if b:
        assert O.bp4x_num_bits(v | np.uint32(1 << (b - 1))) == b


def test_bp4x_sorted_delta():
    v = np.cumsum(np.random.default_rng(1).integers(0, 50, 128)).astype(np.uint32) + 1000
    b = O.bp4x_num_bits(v)
    d = O.bp4x_pack(v, b, sorted_initial=999)
    assert (O.bp4x_unpack(d, b, sorted_initial=999) == v).all()
    deltas = np.diff(np.concatenate([[999], v.astype(np.int64)])).astype(np.uint32)
    assert d == O.bp4x_pack(deltas, b)


def test_roaring_kat():
    exp = bytes.fromhex("3a300000" "02000000" "0000" "0100" "0100" "0000" "18000000" "1c000000" "0100" "0500" "0100")
    assert O.roaring_encode([1, 5, 65537]) == exp
    assert list(O.roaring_decode(exp)) == [1, 5, 65537]


def test_roaring_bitmap_and_run_containers():
    pos = np.arange(0, 20000, 3, dtype=np.uint32)  # 6667 > 4096 -> bitmap container
    enc = O.roaring_encode(pos)
    assert len(enc) == 8 + 8 + 8192
    assert (O.roaring_decode(enc) == pos).all()
    # cookie 12347 with one run container [10, 14] (format spec; not written by roaring 0.10.1)
    run = (12347 | (0 << 16)).to_bytes(4, "little") + b"\x01" + (10).to_bytes(2, "little") + (4).to_bytes(2, "little")
    run = (12347).to_bytes(4, "little") + b"\x01" + (0).to_bytes(2, "little") + (4).to_bytes(2, "little") \
        + (1).to_bytes(2, "little") + (10).to_bytes(2, "little") + (4).to_bytes(2, "little")
    assert list(O.roaring_decode(run)) == [10, 11, 12, 13, 14]


def test_validity_encode_bool_kat():
    v = [True, False, True, True, False, False, False, False, True]
    assert O.write_validity(v) == bytes.fromhex("03000000" "05" "0d01")
    got, pos = O.read_validity(O.write_validity(v), 9)
    assert list(got) == v and pos == 7


def test_validity_rejects_rle_runs():
    # def levels as an RLE run: read_basic.rs:59 unreachable!() -> error
    page = (2).to_bytes(4, "little") + bytes([9 << 1, 1])
    with pytest.raises(O.OracleError):
        O.read_validity(page, 9)


def test_hybrid_rle_mixed_runs():
    # RLE run of 5 x value 3 (bw 2), then a bit-packed group of 8 values
    vals = [1, 2, 3, 0, 1, 2, 3, 0]
    packed = 0
    for i, x in enumerate(vals):
        packed |= x << (2 * i)
    stream = bytes([5 << 1, 3]) + bytes([(1 << 1) | 1]) + packed.to_bytes(2, "little")
    assert list(O.hybrid_decode(stream, 2, 13)) == [3] * 5 + vals


def test_boolean_pages_roundtrip_and_encoder_parity():
    """compress_boolean (boolean/mod.rs:22-61) restated twice -- oracle and
    product encoder -- must agree byte for byte; decode round-trips the valid
    slots (RLE / OneValue drop the bits under nulls, as the reference does)."""
    import pa_amd

    rng = np.random.default_rng(5)
    seen = set()
    for n in [0, 1, 9, 1000, 9000]:
        for v in [rng.random(n) > 0.5, np.repeat(rng.random(n // 64 + 1) > 0.5, 64)[:n], np.ones(n, bool)]:
            valid = rng.random(n) > 0.2
            for kw in [dict(), dict(default_compress_ratio=1.2), dict(default_compression=1), dict(forced_codec=10)]:
                for nullable in [False, True]:
                    opts = pa_amd.WriteOptions(max_page_size=1001, seed=9, **kw)
                    chunk, metas = pa_amd.encode_column(v, valid if nullable else None, nullable, opts)
                    ob, row = b"", 0
                    for i, m in enumerate(metas):
                        oo = O.WriteOptions.make(default_codec=kw.get("default_compression", 0),
                                                 ratio=kw.get("default_compress_ratio"),
                                                 forced=kw.get("forced_codec", -1), seed=pa_amd.page_seed(9, i))
                        pg = O.write_bool_page(v, valid[row:row + m.num_values] if nullable else None, nullable, oo,
                                               offset=row, n=m.num_values)
                        seen.add(pg[(len(O.write_validity(valid[row:row + m.num_values])) if nullable else 0)])
                        ob += pg
                        row += m.num_values
                    assert ob == chunk
                    gv, gm = O.read_bool_column(chunk, [(m.length, m.num_values) for m in metas], nullable)
                    mask = valid if nullable else np.ones(n, bool)
                    assert (gv[mask] == v[mask]).all()
                    if nullable:
                        assert (gm == valid).all()
    assert {O.NONE, O.LZ4, O.RLE, O.ONE_VALUE} <= seen


def test_boolean_basic_keeps_parent_bytes():
    """bitmap.as_slice() of a slice at a byte-aligned offset carries the next
    rows' bits in its last byte (boolean/mod.rs:35-46); unaligned slices are
    rebuilt zero-padded."""
    v = np.array([1, 0, 1, 1, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1], bool)
    pg = O.write_bool_page(v, None, False, O.WriteOptions.make(), offset=0, n=3)
    assert pg[9:] == bytes([0b00001101])
    pg = O.write_bool_page(v, None, False, O.WriteOptions.make(), offset=1, n=3)
    assert pg[9:] == bytes([0b110])
