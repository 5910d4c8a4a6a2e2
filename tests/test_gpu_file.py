"""File -> HBM -> Arrow on the GPU: StrawboatFile reads the footer and the
schema, uploads each column chunk through the pinned double-buffered
pipeline (sb_file_upload) and plans the decoder its leaf type calls for;
every column is compared with the oracle's read of the same chunk.  A
column larger than the two 16 MiB staging buffers cycles both."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
pa = pytest.importorskip("pyarrow")


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _m(metas):
    return [(m.length, m.num_values) for m in metas]


def test_file_mixed_columns(gpu, tmp_path):
    import pa_amd

    rng = np.random.default_rng(11)
    n = 30000
    opts = pa_amd.WriteOptions(default_compress_ratio=1.2, max_page_size=4096)
    a = rng.integers(0, 5000, n).astype(np.int32)
    av = rng.random(n) > 0.2
    b = np.round(rng.normal(0, 100, n), 2)
    strs = [str(x).encode() for x in rng.integers(0, 10**6, n)]
    svals, soffs = pa_amd.binary.strings_to_arrow(strs)
    sv = rng.random(n) > 0.1
    lens = rng.integers(0, 4, n)
    loffs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    child = rng.integers(-99, 99, int(loffs[-1])).astype(np.int64)
    cols = [pa_amd.encode_column(a, av, True, opts),
            pa_amd.encode_column(b, None, False, pa_amd.WriteOptions(default_compression=1, max_page_size=4096)),
            pa_amd.encode_binary_column(svals, soffs, sv, True, opts),
            pa_amd.encode_list_column(loffs, child, None, None, False, False, opts)]
    schema = pa.schema([pa.field("a", pa.int32(), True), pa.field("b", pa.float64(), False),
                        pa.field("s", pa.utf8(), True), pa.field("l", pa.list_(pa.field("item", pa.int64(), False)), False)])
    p = tmp_path / "mixed.sb"
    p.write_bytes(pa_amd.assemble_file(cols, schema.serialize().to_pybytes()[8:]))
    with pa_amd.StrawboatFile(p) as f:
        assert [l.name for l in f.leaves] == ["a", "b", "s", "item"]
        decs = [f.decoder(c) for c in range(4)]  # uploads overlap the plans / decodes before them
        v, m = decs[0].decode()
        ev, em = O.read_column(cols[0][0], _m(cols[0][1]), np.int32, True)
        assert v.cpu().numpy().tobytes() == ev.tobytes()
        assert (pa_amd.unpack_bitmap(m, n).cpu().numpy() == em).all()
        v, _ = decs[1].decode()
        ev, _ = O.read_column(cols[1][0], _m(cols[1][1]), np.float64)
        assert v.cpu().numpy().tobytes() == ev.tobytes()
        o, vals, m = decs[2].decode()
        eo, evals, em = O.read_binary_column(cols[2][0], _m(cols[2][1]), True)
        assert (o.cpu().numpy() == eo).all()
        assert vals.cpu().numpy()[:len(evals)].tobytes() == evals
        assert (pa_amd.unpack_bitmap(m, n).cpu().numpy() == em).all()
        o, _, vals, _ = decs[3].decode()
        eo, _, evals, _ = O.read_list_column(cols[3][0], _m(cols[3][1]), np.int64, False, False)
        assert (o.cpu().numpy() == eo).all()
        assert (vals[:len(evals)].cpu().numpy() == evals).all()


@pytest.mark.parametrize("rows", [1, 6_000_000])  # 48 MB: three staging chunks
def test_file_large_column_pipeline(gpu, tmp_path, rows):
    import pa_amd

    rng = np.random.default_rng(rows)
    x = rng.integers(-(1 << 62), 1 << 62, rows, dtype=np.int64)
    chunk, metas = pa_amd.encode_column(x, None, False, pa_amd.WriteOptions(max_page_size=8192))
    p = tmp_path / "big.sb"
    p.write_bytes(pa_amd.assemble_file([(chunk, metas)], pa.schema([pa.field("x", pa.int64(), False)]).serialize()
                                       .to_pybytes()[8:]))
    with pa_amd.StrawboatFile(p) as f:
        d = f.upload(0)
        torch.cuda.synchronize()
        assert d[:len(chunk)].cpu().numpy().tobytes() == chunk
        v, _ = f.decoder(0, chunk=d).decode()
        assert (v.cpu().numpy() == x).all()


def test_file_leaf_without_page_path(gpu, tmp_path):
    import pa_amd

    chunk, metas = pa_amd.encode_column(np.arange(10, dtype=np.int64), None, True)
    schema = pa.schema([pa.field("dec", pa.decimal128(9, 2), True)])
    p = tmp_path / "dec.sb"
    p.write_bytes(pa_amd.assemble_file([(chunk, metas)], schema.serialize().to_pybytes()[8:]))
    with pa_amd.StrawboatFile(p) as f:
        with pytest.raises(pa_amd.StrawboatError):
            f.decoder(0)
