"""Per-column device encode and decode times of the C5 table (bench.py
WorkloadC5 shapes): which columns dominate.  usage: python tools/c5prof.py [rows]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import torch

    import pa_amd as pa

    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8_388_608
    W = bench.WorkloadC5
    rng = np.random.default_rng(555)
    specs = ([(np.int32, k) for k in W.I32] + [(np.int64, k) for k in W.I64] + [(np.float64, k) for k in W.F64] +
             [("utf8", k) for k in W.STR] + [(np.bool_, k) for k in W.BOOL] + [(np.uint32, k) for k in W.U32])
    ctx = pa.default_context(0)
    res = []
    for ci, (dt, kind) in enumerate(specs):
        nullable = dt != "utf8" and ci % 4 == 3
        valid = (rng.random(rows) >= 0.1) if nullable else None
        basic = kind in ("lz4", "none")
        opts = pa.WriteOptions(default_compression=1 if kind == "lz4" else 0,
                               default_compress_ratio=None if basic else 2.0, max_page_size=bench.PAGE_ROWS, seed=555 + ci)
        if dt == "utf8":
            svals, soffs = W._strings(kind, rows, rng)
            tv = torch.from_numpy(np.frombuffer(svals, np.uint8).copy()).cuda()
            to = torch.from_numpy(soffs).cuda()
            enc = lambda: pa.encode_binary_column_device(tv, to, None, False, opts, pa.UTF8, ctx=ctx)  # noqa: E731
        else:
            v = W._values(dt, kind, rows, rng)
            tv = torch.from_numpy(v).cuda()
            tvalid = None if valid is None else torch.from_numpy(valid).cuda()
            enc = lambda: pa.encode_column_device(tv, tvalid, nullable, opts, ctx=ctx)  # noqa: E731
        chunk, metas = enc()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            chunk, metas = enc()
        torch.cuda.synchronize()
        te = (time.perf_counter() - t0) / 3
        if dt == "utf8":
            dec = pa.BinaryColumnDecoder(chunk, metas, pa.UTF8, False, ctx=ctx)
        else:
            dec = pa.ColumnDecoder(chunk, metas, dt, nullable, ctx=ctx)
        outs = dec.alloc_outputs()
        dec.decode(*outs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            dec.decode_async(*outs)
        torch.cuda.synchronize()
        td = (time.perf_counter() - t0) / 5
        mix = bench.page_codecs(chunk.cpu().numpy().tobytes(), metas, nullable)
        res.append((te, td, ci, str(dt), kind, nullable, mix))
        print(f"col {ci:2d} {str(dt):28s} {kind:7s} null={int(nullable)} enc {te*1e3:8.2f} ms dec {td*1e3:7.3f} ms {mix}",
              flush=True)
    print("total enc %.1f ms dec %.1f ms" % (sum(r[0] for r in res) * 1e3, sum(r[1] for r in res) * 1e3))


if __name__ == "__main__":
    main()
