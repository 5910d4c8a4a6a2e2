"""Replays test_int_columns[null-force_dict-uint16] and prints mismatches."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import oracle as O
from tests.colgen import build_column, gen_values, oracle_decode_column
import pa_amd
ctx = pa_amd.default_context(0)
rng = np.random.default_rng(42)
dtype = np.uint16
for kind in ["index", "full", "sorted", "one", "runs", "short_runs", "freq"]:
    n = 20000
    values = gen_values(kind, n, dtype, rng)
    validity = rng.random(n) > 0.2
    opts = O.WriteOptions.make(forbidden=(O.PATAS,), ratio=2.0, forced=O.DICT)
    for page_rows in (2048, 8192):
        chunk, metas, codecs = build_column(values, validity, True, page_rows, opts)
        ov, om = oracle_decode_column(chunk, metas, dtype, True)
        dec = pa_amd.ColumnDecoder(chunk, [pa_amd.PageMeta(l, m) for l, m in metas], dtype, True, ctx)
        v, bm = dec.decode()
        gv = v.cpu().numpy().view(np.uint16)[:n]
        bmh = bm.cpu().numpy()
        gm = np.unpackbits(bmh, bitorder="little")[:n].astype(bool)
        bad = np.nonzero(gm != om)[0]
        badv = np.nonzero(gv != ov)[0]
        print(kind, page_rows, "codecs", set(codecs), "val-bad", len(badv), "valid-bad", len(bad), bad[:10], "bm bytes", len(bmh), "vals bytes", v.numel()*2)
        if len(bad):
            print("  rows", bad[:5], "gm", gm[bad[:5]], "om", om[bad[:5]], "bytes", bmh[bad[0]//8 - 2: bad[0]//8 + 4])
