"""Per-unit kernel times from a kernel trace of tools/c5units.py:
python tools/unit_kernels.py <kernel_trace.csv> <c5units.log>
Dispatch clusters separated by > 5 ms are the solo decodes, 5 per unit in
the log's order (after the encode and set-up traffic); prints each unit's
median kernel times."""
import collections
import csv
import re
import sys

import numpy as np


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    units = [l for l in open(sys.argv[2]) if re.match(r"^(ColumnGroupDecoder|BinaryColumnDecoder)", l)]
    cl, cur, last = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last is not None and s - last > 5_000_000:
            cl.append(cur)
            cur = []
        cur.append((r["Kernel_Name"], s, e))
        last = max(last or 0, e)
    cl.append(cur)
    need = 5 * len(units)
    # the solo decodes are the last `need` clusters before the 4-stream step run
    # solo decodes: clusters of engine kernels only (the bench's verify runs
    # torch kernels; its steps launch far more dispatches), the last `need`
    solo = [c for c in cl if len(c) < 120 and all(k.startswith(("sbk::", "void sbk::", "__amd_rocclr")) for k, _, _ in c)]
    solo = solo[-need:]
    for i, u in enumerate(units):
        reps = solo[5 * i:5 * i + 5][1:]
        per = collections.defaultdict(list)
        for c in reps:
            acc = collections.defaultdict(float)
            for k, s, e in c:
                acc[k] += (e - s) / 1e3
            for k, v in acc.items():
                per[k].append(v)
            per["(span)"].append((max(e for _, _, e in c) - min(s for _, s, _ in c)) / 1e3)
        print(u.strip())
        for k, v in sorted(per.items(), key=lambda kv: -np.median(kv[1])):
            if np.median(v) >= 2:
                print(f"    {np.median(v):9.1f} us  {k[:90]}")


if __name__ == "__main__":
    main()
