"""Per-kernel summaries for profiles/: python tools/prof_summary.py trace <kernel_trace.csv> <steps> <out.json>
(avg duration per kernel over the last `steps` step's worth of dispatches, and
dispatches per step) or pmc <fetch_csv> <write_csv> <out.json> (HBM bytes per
dispatch per kernel, MI355X_MICROARCH.md's gfx950 corrections: fetch = 2 x
FETCH_SIZE x 1 KiB, write = WRITE_SIZE x 1 KiB; first dispatch of each kernel
skipped as cold)."""
import collections
import csv
import json
import sys


def trace(path, steps, out):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for k, d in by.items():
        res[k[:120]] = {"dispatches": len(d), "avg_us": round(sum(d) / len(d), 2),
                        "avg_us_last": round(sum(d[-max(1, len(d) // 2):]) / max(1, len(d) // 2), 2),
                        "total_us": round(sum(d), 1)}
    res = dict(sorted(res.items(), key=lambda kv: -kv[1]["total_us"]))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1)[:3000])


def pmc(fpath, wpath, out):
    def per(path, counter):
        v = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == counter:
                v[r["Kernel_Name"][:120]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        return v

    f, w = per(fpath, "FETCH_SIZE"), per(wpath, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fv = [x for _, x in sorted(f[k].items())]
        wv = [x for _, x in sorted(w[k].items())]
        fv, wv = fv[1:] or fv, wv[1:] or wv
        fb = 2.0 * 1024 * sum(fv) / max(1, len(fv))
        wb = 1024 * sum(wv) / max(1, len(wv))
        res[k] = {"fetch_bytes_per_dispatch": int(fb), "write_bytes_per_dispatch": int(wb),
                  "hbm_bytes_per_dispatch": int(fb + wb), "dispatches": [len(fv), len(wv)],
                  "raw_fetch_kib": round(sum(fv) / max(1, len(fv)), 1), "raw_write_kib": round(sum(wv) / max(1, len(wv)), 1)}
    res["_correction"] = "fetch = 2 x FETCH_SIZE x 1KiB (gfx950 16 B/lane read undercount), write = WRITE_SIZE x 1KiB"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(sys.argv[2], int(sys.argv[3]), sys.argv[4])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4])
