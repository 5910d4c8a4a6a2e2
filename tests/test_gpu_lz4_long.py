"""LZ4 / Snappy pages whose literals span many ring chunks: the body of a
long literal is copied straight to the column (k_inflate lit_global), so
matches after it that reach back into that body read it from HBM.  Pages:
random bytes followed by copies of earlier parts at offsets up to the 64 KiB
LZ4 window, checked against the oracle (liblz4 / snappy via basic.rs)."""
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


def pages(rng, n):
    """Rows of int64: a random head, then back-references of several reaches."""
    head = rng.integers(-2**63, 2**63 - 1, n // 2, dtype=np.int64)
    tail = []
    while sum(len(t) for t in tail) < n - len(head):
        a = int(rng.integers(0, len(head) - 64))
        tail.append(head[a:a + int(rng.integers(1, 64))])
        tail.append(rng.integers(-2**63, 2**63 - 1, int(rng.integers(0, 3)), dtype=np.int64))
    return np.concatenate([head] + tail)[:n]


@pytest.mark.parametrize("codec", [1, 3], ids=["lz4", "snappy"])
@pytest.mark.parametrize("nullable", [False, True], ids=["req", "null"])
@pytest.mark.parametrize("page_rows", [700, 2000, 8192])
def test_long_literals(ctx, codec, nullable, page_rows):
    import pa_amd

    rng = np.random.default_rng(page_rows + codec)
    v = np.concatenate([pages(rng, page_rows) for _ in range(6)])
    valid = rng.random(len(v)) > 0.1 if nullable else None
    chunk, metas = pa_amd.encode_column(v, valid, nullable,
                                        pa_amd.WriteOptions(default_compression=codec, max_page_size=page_rows))
    got, gm = pa_amd.ColumnDecoder(chunk, metas, np.int64, nullable, ctx).decode()
    ev, em = O.read_column(chunk, [(m.length, m.num_values) for m in metas], np.int64, nullable)
    assert got.cpu().numpy().tobytes() == ev.tobytes()
    if nullable:
        assert (pa_amd.read.unpack_bitmap(gm, len(v)).cpu().numpy() == em).all()
