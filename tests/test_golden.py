"""Golden page fixtures (tests/golden/pages.npz, tools/gen_golden.py):
the oracle decodes each committed page to its committed values and the
product's host encoder writes the committed bytes again (fixed seed)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pages.npz")


def cases():
    z = np.load(GOLD)
    keys = sorted({k.split("__")[0] for k in z.files})
    for k in keys:
        yield k, z


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _parse(key):
    dtype, null, name = key.split("_", 2)
    return np.dtype(dtype), null == "null", name


def test_golden_oracle_decode(gold):
    keys = sorted({k.split("__")[0] for k in gold.files})
    assert len(keys) > 100
    for k in keys:
        dt, nullable, _ = _parse(k)
        page = gold[k + "__page"].tobytes()
        exp = gold[k + "__values"]
        vals, vv = O.read_page(page, len(exp), dt, nullable)
        assert vals.tobytes() == exp.tobytes(), k
        if nullable:
            assert (vv == gold[k + "__validity"]).all(), k


def test_golden_product_encoder_reproduces_bytes(gold):
    import pa_amd

    keys = sorted({k.split("__")[0] for k in gold.files})
    for k in keys:
        dt, nullable, name = _parse(k)
        if dt == np.float32 and name == "patas":
            continue
        cname = name.split("_")[-1] if "_" in name else ""
        base = name.split("_")[0]
        dc = {"lz4": 1, "zstd": 2, "snappy": 3}.get(cname, 0)
        kw = {"plain": dict(default_compress_ratio=None), "adaptive": dict(default_compress_ratio=1.2),
              "rle": dict(default_compress_ratio=1.0, forced_codec=O.RLE),
              "dict": dict(default_compress_ratio=1.0, forced_codec=O.DICT),
              "freq": dict(default_compress_ratio=1.0, forced_codec=O.FREQ),
              "bitpacking": dict(default_compress_ratio=0.001, forced_codec=O.BITPACKING),
              "patas": dict(default_compress_ratio=1.0, forced_codec=O.PATAS)}[base]
        data = gold[k + "__input"]
        valid = gold[k + "__validity"] if nullable else None
        # the fixture's validity is the decoded one == the written one
        page = pa_amd.encode_page(data, valid, nullable, pa_amd.WriteOptions(default_compression=dc, seed=7, **kw))
        assert page == gold[k + "__page"].tobytes(), k
