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


# ---- the non-fixed-width families (tests/golden/columns.npz) ---------------
from tests import goldcols as G  # noqa: E402


@pytest.fixture(scope="module")
def gcols():
    return G.load()


def _bits(t, n):
    return np.unpackbits(t.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)


def test_golden_binary_columns(ctx, gcols):
    """Utf8 / LargeBinary chunks under None / LZ4 / Zstd / Snappy, Dict, Freq,
    OneValue and the adaptive choice through BinaryColumnDecoder, byte for
    byte: offsets, values, validity (read_binary, binary.rs:223-265)."""
    import pa_amd

    cases = G.cases(gcols, "bin_")
    assert len(cases) == 36
    for case in cases:
        kind, null = case.split("_")[1:3]
        phys = pa_amd.LARGE_BINARY if kind == "largebin" else pa_amd.UTF8
        metas = [pa_amd.PageMeta(l, n) for l, n in G.metas(gcols, case)]
        dec = pa_amd.BinaryColumnDecoder(gcols[case + "__chunk"], metas, phys, null == "null", ctx)
        o, v, m = dec.decode()
        n, vb = dec.num_rows, dec.values_bytes
        dec.close()
        assert (o.cpu().numpy().astype(np.int64)[: n + 1] == gcols[case + "__offsets"]).all(), case
        assert v.cpu().numpy()[:vb].tobytes() == gcols[case + "__values"].tobytes(), case
        if null == "null":
            assert (_bits(m, n) == gcols[case + "__validity"]).all(), case


def test_golden_bool_columns(ctx, gcols):
    """Boolean chunks (Basic under each general codec at byte-aligned and
    ragged page offsets, RLE, OneValue) through the Boolean column decoder
    (read_boolean, boolean.rs:191-219)."""
    import pa_amd

    cases = G.cases(gcols, "bool_")
    assert len(cases) == 18
    for case in cases:
        nullable = case.split("_")[1] == "null"
        metas = [pa_amd.PageMeta(l, n) for l, n in G.metas(gcols, case)]
        dec = pa_amd.ColumnDecoder(gcols[case + "__chunk"], metas, np.bool_, nullable, ctx)
        v, m = dec.decode()
        n = dec.num_rows
        dec.close()
        assert (_bits(v, n) == gcols[case + "__values"]).all(), case
        if nullable:
            assert (_bits(m, n) == gcols[case + "__validity"]).all(), case


def test_golden_list_i32_columns(ctx, gcols):
    """List<Int32> chunks through ListColumnDecoder (create_list, list.rs:48):
    offsets, list validity, every leaf value (under nulls too), leaf validity."""
    import pa_amd

    cases = G.cases(gcols, "nest_list_i32")
    assert len(cases) == 4
    for case in cases:
        f = G.field(gcols, case)
        ((chunk, metas), exp), = G.leaf_reads(gcols, case, f)
        dec = pa_amd.ListColumnDecoder(chunk, [pa_amd.PageMeta(l, n) for l, n in metas], np.int32, True, True, ctx)
        go, gl, gv, gf = dec.decode()
        rows, leaves = dec.num_rows, dec.num_leaves
        dec.close()
        assert (go.cpu().numpy().astype(np.int64) == exp["offsets"][0]).all(), case
        assert (_bits(gl, rows) == exp["validity"][0]).all(), case
        assert gv.cpu().numpy().view(np.int32)[:leaves].tobytes() == exp["values"].tobytes(), case
        assert (_bits(gf, leaves) == exp["leaf_validity"]).all(), case


def test_golden_nested_fields(ctx, gcols):
    """List<Int32>, List<Utf8>, Struct<LargeBinary, Int32, Boolean> and
    Map<Int32, Utf8> chunks through FieldDecoder, assembled and compared with
    the committed per-leaf reads assembled the same way (values under nulls
    included)."""
    import pa_amd

    from oracle import nest as NE
    from tests import nestgen

    cases = G.cases(gcols, "nest_")
    assert len(cases) == 16
    for case in cases:
        f = G.field(gcols, case)
        leaves = G.leaf_reads(gcols, case, f)
        cols = [(c, [pa_amd.PageMeta(l, n) for l, n in m]) for (c, m), _ in leaves]
        dec = pa_amd.FieldDecoder(nestgen.pa_amd_field(f), cols, ctx)
        try:
            got = nestgen.device_to_host(f, dec.decode())
        finally:
            dec.close()
        NE.equal(f, got, NE.assemble(f, [e for _, e in leaves]), values_under_nulls=True)
