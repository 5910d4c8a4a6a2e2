"""Sharded decode on one GPU: the chunk's page ranges for
2 and 3 ranks are decoded one after the other by ColumnDecoder /
BinaryColumnDecoder / ListColumnDecoder .for_shard, placed with the host-side
scans (exclusive_bases of the shards' value bytes / leaf counts / rows), and
must reassemble bit-exactly into the whole column -- compared with the
oracle's whole-column read and with pa_amd's own whole-column decode."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.test_shard_gloo import _columns

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def cols():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _columns()


@pytest.mark.parametrize("world", [2, 3])
def test_flat_shards(cols, world):
    import pa_amd

    chunk, metas = cols[0]
    d = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda()
    whole, _ = pa_amd.ColumnDecoder(d, metas, np.int32, False).decode()
    out = torch.empty_like(whole)
    for sh in pa_amd.shard_pages(metas, world):
        v, _ = pa_amd.ColumnDecoder.for_shard(d, metas, sh, np.int32, False).decode()
        out[sh.row_offset:sh.row_offset + sh.rows] = v[:sh.rows]
    assert torch.equal(out, whole)
    assert (out.cpu().numpy() == O.read_column(chunk, [(m.length, m.num_values) for m in metas], np.int32)[0]).all()


@pytest.mark.parametrize("world", [2, 3])
def test_utf8_shards(cols, world):
    import pa_amd

    chunk, metas = cols[1]
    d = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda()
    decs = [pa_amd.BinaryColumnDecoder.for_shard(d, metas, sh, pa_amd.UTF8, True) for sh in pa_amd.shard_pages(metas, world)]
    bases = pa_amd.exclusive_bases([dc.values_bytes for dc in decs])
    offs, vals, valid = [], [], []
    for dc, b in zip(decs, bases):
        o, v, m = dc.decode()
        offs.append(pa_amd.rebase_offsets(o.long(), b)[(1 if offs else 0):])
        vals.append(v[:dc.values_bytes])
        valid.append(pa_amd.read.unpack_bitmap(m, dc.num_rows))
    eo, ev, em = O.read_binary_column(chunk, [(m.length, m.num_values) for m in metas], True)
    assert (torch.cat(offs).cpu().numpy() == eo).all()
    assert torch.cat(vals).cpu().numpy().tobytes() == ev
    assert (torch.cat(valid).cpu().numpy() == em).all()


@pytest.mark.parametrize("world", [2, 3])
def test_list_shards(cols, world):
    import pa_amd

    chunk, metas = cols[2]
    d = torch.from_numpy(np.frombuffer(chunk, np.uint8).copy()).cuda()
    decs = [pa_amd.ListColumnDecoder.for_shard(d, metas, sh, np.int64, False, False)
            for sh in pa_amd.shard_pages(metas, world)]
    bases = pa_amd.exclusive_bases([dc.num_leaves for dc in decs])
    offs, vals = [], []
    for dc, b in zip(decs, bases):
        o, _, v, _ = dc.decode()
        offs.append(pa_amd.rebase_offsets(o.long(), b)[(1 if offs else 0):])
        vals.append(v[:dc.num_leaves])
    eo, _, ev, _ = O.read_list_column(chunk, [(m.length, m.num_values) for m in metas], np.int64, False, False)
    assert (torch.cat(offs).cpu().numpy() == eo).all()
    assert (torch.cat(vals).cpu().numpy() == ev).all()
