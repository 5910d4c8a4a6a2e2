"""Golden column fixtures for the non-fixed-width families
(tests/golden/columns.npz, tools/gen_golden.py): Binary / Utf8 under every
general codec and Dict / Freq / OneValue (binary/mod.rs:95-183), Boolean
Basic / RLE / OneValue (boolean/mod.rs:63-102), List<Int32>, List<Utf8>,
Struct and Map fields (read_basic.rs:65-173).  The oracle must still decode
each chunk to the committed buffers, and the product's host writer must
write the committed chunk bytes again from the committed inputs (page p
sampled with sb_page_seed(7, p)).  The GPU decode of the same chunks is
tests/test_gpu_golden.py."""
import numpy as np
import pytest

import pa_amd
from oracle import nest as NE
from oracle import oracle as O
from tests import goldcols as G, nestgen

PHYS = {"utf8": pa_amd.UTF8, "largebin": pa_amd.LARGE_BINARY}


@pytest.fixture(scope="module")
def z():
    return G.load()


def test_fixture_covers_every_family(z):
    assert len(G.cases(z, "bin_")) == 36
    assert len(G.cases(z, "bool_")) == 18
    assert len(G.cases(z, "nest_")) == 16


def test_page_seed_restatement():
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("gg", os.path.join(os.path.dirname(__file__), "..", "tools",
                                                                     "gen_golden.py"))
    src = open(spec.origin).read()
    ns = {}
    exec(compile(src[src.index("M64 = "):src.index("SEED = 7")], "gen_golden", "exec"), ns)  # the function only
    for s, p in ((7, 0), (7, 1), (0, 12345), (2 ** 63 + 5, 2 ** 40)):
        assert ns["page_seed"](s, p) == pa_amd.page_seed(s, p)


def _opts(name, dc, step):
    kw = {"plain": dict(), "adaptive": dict(default_compress_ratio=2.0), "onevalue": dict(default_compress_ratio=2.0),
          "rle": dict(default_compress_ratio=1.0, forced_codec=O.RLE),
          "dict": dict(default_compress_ratio=1.0, forced_codec=O.DICT),
          "freq": dict(default_compress_ratio=1.0, forced_codec=O.FREQ)}[name]
    return pa_amd.WriteOptions(default_compression=dc, max_page_size=step, seed=G.SEED, **kw)


def _name_codec(case, skip):
    rest = case.split("_", skip)[-1]
    parts = rest.split("_")
    dc = {"lz4": 1, "zstd": 2, "snappy": 3}.get(parts[1] if len(parts) > 1 else "", 0)
    return parts[0], dc


def test_binary_columns(z):
    for case in G.cases(z, "bin_"):
        _, kind, null, _ = case.split("_", 3)
        nullable = null == "null"
        ow = 8 if kind == "largebin" else 4
        chunk, metas = z[case + "__chunk"].tobytes(), G.metas(z, case)
        eo, ev, evalid = O.read_binary_column(chunk, metas, nullable, ow)
        assert (eo == z[case + "__offsets"]).all() and ev == z[case + "__values"].tobytes(), case
        if nullable:
            assert (evalid == z[case + "__validity"]).all(), case
        name, dc = _name_codec(case, 3)
        got, gm = pa_amd.encode_binary_column(z[case + "__in_values"].tobytes(), z[case + "__in_offsets"],
                                              G.get(z, case + "__in_validity"), nullable, _opts(name, dc, 500),
                                              PHYS[kind])
        assert got == chunk and [(m.length, m.num_values) for m in gm] == metas, case


def test_bool_columns(z):
    for case in G.cases(z, "bool_"):
        nullable = case.split("_")[1] == "null"
        chunk, metas = z[case + "__chunk"].tobytes(), G.metas(z, case)
        ev, evalid = O.read_bool_column(chunk, metas, nullable)
        assert (ev == z[case + "__values"]).all(), case
        if nullable:
            assert (evalid == z[case + "__validity"]).all(), case
        name, dc = _name_codec(case, 2)
        got, gm = pa_amd.encode_column(z[case + "__in_values"], G.get(z, case + "__in_validity"), nullable,
                                       _opts(name, dc, int(z[case + "__step"])))
        assert got == chunk and [(m.length, m.num_values) for m in gm] == metas, case


def test_nested_columns(z):
    for case in G.cases(z, "nest_"):
        f = G.field(z, case)
        leaves = G.leaf_reads(z, case, f)
        for path, ((chunk, metas), exp) in zip(NE.leaf_paths(f), leaves):
            r = NE.read_leaf(path, chunk, metas)
            assert r["counts"] == exp["counts"], case
            NE.equal(path[-1], NE.A("leaf", r["counts"][-1], r["leaf_validity"], values=r["values"]),
                     NE.A("leaf", exp["counts"][-1], exp["leaf_validity"], values=exp["values"]))
        a = G.input_array(z, case, f)
        NE.equal(f, NE.assemble(f, [e for _, e in leaves]), a, values_under_nulls=False)
        dc = {"lz4": 1, "zstd": 2}.get(case.split("_")[-1], 0)
        base = "adaptive" if "adaptive" in case else "plain"
        got = pa_amd.encode_field(nestgen.pa_amd_field(f), nestgen.host_array(a), _opts(base, dc, 500))
        for (gc, gm), ((chunk, metas), _) in zip(got, leaves):
            assert gc == chunk and [(m.length, m.num_values) for m in gm] == metas, case
