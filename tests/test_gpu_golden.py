"""GPU parity on the committed golden pages (tests/golden/pages.npz, made by
tools/gen_golden.py): every page decodes through the C ABI
(sb_plan_column + sb_decode_planned via pa_amd.ColumnDecoder) to the
fixture's `__values` bytes (null slots included) and `__validity` bits.

Two shapes: each page alone as a one-page column chunk, and every page of one
(type, nullability) back to back as one column with mixed codecs, so a page's
row base and validity bit offset are not always 0 (read/array/integer.rs:
210-238 appends pages in order)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pages.npz")


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pa_amd

    return pa_amd.default_context(0)


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _keys(gold):
    return sorted({k.split("__")[0] for k in gold.files})


def _parse(key):
    dtype, null, name = key.split("_", 2)
    return np.dtype(dtype), null == "null", name


def _decode(ctx, pages, dtype, nullable):
    import pa_amd

    chunk = np.frombuffer(b"".join(p for p, _ in pages), np.uint8)
    metas = [pa_amd.PageMeta(len(p), n) for p, n in pages]
    dec = pa_amd.ColumnDecoder(chunk, metas, dtype, nullable, ctx)
    vals, bm = dec.decode()
    n = dec.num_rows
    v = vals.cpu().numpy().view(np.uint8)[: n * dtype.itemsize].view(dtype)
    valid = None
    if nullable:
        valid = np.unpackbits(bm.cpu().numpy(), bitorder="little")[:n].astype(bool)
    dec.close()
    return v, valid


def test_golden_pages_one_by_one(ctx, gold):
    keys = _keys(gold)
    assert len(keys) > 100
    for k in keys:
        dt, nullable, _ = _parse(k)
        page = gold[k + "__page"].tobytes()
        exp = gold[k + "__values"]
        v, vv = _decode(ctx, [(page, len(exp))], dt, nullable)
        assert v.view(np.uint8).tobytes() == exp.view(np.uint8).tobytes(), k
        if nullable:
            assert (vv == gold[k + "__validity"]).all(), k


def test_golden_pages_as_mixed_columns(ctx, gold):
    groups = {}
    for k in _keys(gold):
        dt, nullable, _ = _parse(k)
        groups.setdefault((dt.str, nullable), []).append(k)
    assert len(groups) == 14
    for (dts, nullable), ks in groups.items():
        dt = np.dtype(dts)
        # in order, then reversed behind a 37-row plain page the oracle writes,
        # so every golden page also decodes at a row / bit offset = 5 mod 32
        lead = np.arange(37).astype(dt)
        lead_valid = (np.arange(37) % 3 != 0) if nullable else None
        lead_page = O.write_page(lead, lead_valid, nullable, O.WriteOptions.make(ratio=None))
        for order, pre in ((ks, []), (ks[::-1], [(lead_page, 37, lead, lead_valid)])):
            pages = [(p, n) for p, n, _, _ in pre]
            pages += [(gold[k + "__page"].tobytes(), len(gold[k + "__values"])) for k in order]
            v, vv = _decode(ctx, pages, dt, nullable)
            exp = np.concatenate([x for _, _, x, _ in pre] + [gold[k + "__values"] for k in order])
            assert v.view(np.uint8).tobytes() == exp.view(np.uint8).tobytes(), (dts, nullable)
            if nullable:
                ev = np.concatenate([x for _, _, _, x in pre] + [gold[k + "__validity"] for k in order])
                assert (vv == ev).all(), (dts, nullable)
