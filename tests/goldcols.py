"""Loader of tests/golden/columns.npz (tools/gen_golden.py): the committed
non-fixed-width column chunks -- Binary / Utf8, Boolean, List<Int32>,
List<Utf8>, Struct and Map fields -- with the inputs they were written from
and the Arrow buffers the oracle decoded them to."""
from __future__ import annotations

import json
import os

import numpy as np

from oracle import nest as NE

GOLD = os.path.join(os.path.dirname(__file__), "golden", "columns.npz")
SEED = 7


def load():
    return np.load(GOLD)  # allow_pickle=False: plain arrays only


def cases(z, prefix):
    return sorted({k.split("__")[0] for k in z.files if k.startswith(prefix)})


def get(z, key):
    return z[key] if key in z.files else None


def metas(z, case):
    return [(int(l), int(n)) for l, n in z[case + "__metas"]]


def field(z, case) -> NE.F:
    def mk(d):
        return NE.F(d["kind"], d["nullable"], [mk(c) for c in d["children"]], leaf=d["leaf"],
                    dtype=None if d["dtype"] is None else np.dtype(d["dtype"]), large=d["large"], name=d["name"])
    return mk(json.loads(str(z[case + "__field"])))


def input_array(z, case, f: NE.F) -> NE.A:
    """The written array, rebuilt from its pre-order nodes."""
    it = iter(range(10 ** 6))

    def mk(fx):
        i = next(it)
        p = f"{case}__node{i}__"
        n = int(z[p + "length"])
        v = get(z, p + "validity")
        if fx.kind == "leaf":
            vals = z[p + "values"]
            if fx.leaf == "binary":
                vals = (z[p + "values_offsets"], vals.tobytes())
            return NE.A("leaf", n, v, values=vals)
        return NE.A(fx.kind, n, v, offsets=get(z, p + "offsets"), children=[mk(c) for c in fx.children])
    return mk(f)


def leaf_reads(z, case, f: NE.F):
    """Per leaf column: (chunk, metas) and the oracle's read_leaf dict."""
    out = []
    for k, path in enumerate(NE.leaf_paths(f)):
        p = f"{case}__{k}__"
        D = len(path) - 1
        vals = z[p + "values"]
        if path[-1].leaf == "binary":
            vals = (z[p + "values_offsets"], vals.tobytes())
        r = dict(offsets=[get(z, p + f"offsets{d}") for d in range(D)],
                 validity=[get(z, p + f"validity{d}") for d in range(D)], values=vals,
                 leaf_validity=get(z, p + "leaf_validity"), counts=[int(x) for x in z[p + "counts"]])
        out.append(((z[p + "chunk"].tobytes(), [(int(l), int(n)) for l, n in z[p + "metas"]]), r))
    return out
