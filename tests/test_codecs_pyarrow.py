"""General codecs (compression/basic.rs:62-152) cross-checked against
independent implementations: pyarrow's lz4_raw / zstd / snappy codecs."""
import numpy as np
import pytest

from oracle import oracle as O

pa = pytest.importorskip("pyarrow")

CODECS = [(O.LZ4, "lz4_raw"), (O.ZSTD, "zstd"), (O.SNAPPY, "snappy")]


def payloads():
    rng = np.random.default_rng(0)
    yield b""
    yield b"a"
    yield bytes(range(256)) * 40
    yield rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    yield np.round(rng.standard_normal(8192) * 1e4, 2).tobytes()
    yield np.repeat(rng.integers(0, 100, 300), 37).astype(np.int32).tobytes()


@pytest.mark.parametrize("codec,name", CODECS, ids=[c[1] for c in CODECS])
def test_oracle_compress_decodes_with_pyarrow(codec, name):
    c = pa.Codec(name)
    for data in payloads():
        enc = O.common_compress(codec, data)
        assert c.decompress(enc, decompressed_size=len(data)).to_pybytes() == data


@pytest.mark.parametrize("codec,name", CODECS, ids=[c[1] for c in CODECS])
def test_pyarrow_compress_decodes_with_oracle(codec, name):
    c = pa.Codec(name)
    for data in payloads():
        if not data and name == "lz4_raw":
            continue
        enc = c.compress(data, asbytes=True)
        assert O.common_decompress(codec, enc, len(data)) == data


def test_corrupt_streams_error():
    data = bytes(range(200)) * 50
    for codec, _ in CODECS:
        enc = bytearray(O.common_compress(codec, data))
        enc = enc[: len(enc) // 2]
        with pytest.raises(O.OracleError):
            O.common_decompress(codec, bytes(enc), len(data))
