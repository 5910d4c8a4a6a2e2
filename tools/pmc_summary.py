"""HBM traffic per decode step from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE in separate runs, MI355X_MICROARCH.md §HBM): python
tools/pmc_summary.py <workload> <fetch_csv> <write_csv> <bytes.json>
<out.json> <commit>.

Correction (calibrated this round, profiles/r03_pmc_calibration.json, 1 GiB
buffers): FETCH_SIZE counts 64 B per memory request of up to 128 B, so
fetch bytes = 2 x FETCH_SIZE KiB for coalesced 16-B, dword and byte loads
alike, and for scattered dword reads it is the 128-B line each request
brings; WRITE_SIZE is exact for 16-B and dword stores (byte stores +0.9 %).

The step window is the dispatches between the last two marker launches
(an int16 arange, tools/wlbench.py): every kernel dispatched there, however
many times per step, is attributed to the `steps` steps.  A k_inflate
dispatch is tagged with the pass before it (fixed-width or binary), so C3's
Float64 and Utf8 streams are reported apart.  `algorithmic` is the workload's
compressed bytes read plus Arrow bytes written per step (bytes.json, from
tools/wlbench.py)."""
import collections
import csv
import json
import os
import sys


def per_dispatch(path, counter):
    v = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d = int(r["Dispatch_Id"])
        v[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return v, names


def tag(names):
    """kernel label per dispatch in the marker window: k_inflate after a
    binary pass is 'k_inflate[binary]'."""
    marks = [d for d in sorted(names) if "arange" in names[d]]
    if len(marks) < 2:
        raise SystemExit("no marker window (run tools/wlbench.py with a bytes.json argument)")
    lo, hi = marks[-2], marks[-1]
    out, prev = {}, ""
    for d in sorted(names):
        if not lo < d < hi:
            continue
        n = names[d].split("(")[0].replace("void ", "")
        if n.endswith("k_inflate"):
            n += "[binary]" if "k_bin" in prev else "[fixed]"
        out[d] = n
        prev = n
    return out


def main():
    wl, fcsv, wcsv, bjson, out, commit = sys.argv[1:7]
    rnd = int(sys.argv[7]) if len(sys.argv) > 7 else int(os.environ.get("SB_ROUND", "6"))
    by = json.load(open(bjson))
    f, fn = per_dispatch(fcsv, "FETCH_SIZE")
    w, wn = per_dispatch(wcsv, "WRITE_SIZE")
    ft, wt = tag(fn), tag(wn)
    steps = int(by.get("steps", 3))
    kernels = {}
    step_f = step_w = 0.0
    fs, ws = collections.defaultdict(list), collections.defaultdict(list)
    for d, k in ft.items():
        fs[k].append(f[d])
    for d, k in wt.items():
        ws[k].append(w[d])
    for k in sorted(set(fs) | set(ws)):
        a, b = fs.get(k, []), ws.get(k, [])
        if len(a) != len(b):
            raise SystemExit(f"{k}: {len(a)} fetch vs {len(b)} write dispatches in the window")
        fb = 2.0 * 1024 * sum(a) / steps
        wb = 1024.0 * sum(b) / steps
        kernels[k] = {"fetch_bytes_per_step": int(fb), "write_bytes_per_step": int(wb),
                      "dispatches_per_step": len(a) / steps}
        step_f += fb
        step_w += wb
    alg = by["in_bytes"] + by["out_bytes"]
    res = {"workload": wl, "commit": commit, "round": rnd,
           "window": f"{steps} steps between two marker launches",
           "correction": "fetch = 2 x FETCH_SIZE x 1 KiB (calibrated, profiles/r03_pmc_calibration.json); "
                         "write = WRITE_SIZE x 1 KiB",
           "algorithmic_bytes_per_step": alg, "in_bytes": by["in_bytes"], "out_bytes": by["out_bytes"],
           "columns": by.get("columns", {}),
           "step": {"fetch_bytes": int(step_f), "write_bytes": int(step_w), "hbm_bytes": int(step_f + step_w),
                    "traffic_over_algorithmic": round((step_f + step_w) / alg, 4)},
           "kernels": kernels}
    cols = by.get("columns", {})
    for k, v in kernels.items():  # per-kernel algorithmic bytes where one kernel carries one column's bytes
        col = None
        if k.startswith("sbk::k_decode_staged") and wl in ("c2", "c2h"):
            col = next(iter(cols.values()))
        elif k == "sbk::k_inflate[fixed]" and "float64" in cols:
            col = cols["float64"]
        elif k == "sbk::k_inflate[binary]" and "utf8" in cols:
            col = cols["utf8"]
        if col:
            a = col["in_bytes"] + col["out_bytes"]
            v["algorithmic_bytes_per_step"] = a
            v["traffic_over_algorithmic"] = round((v["fetch_bytes_per_step"] + v["write_bytes_per_step"]) / a, 4)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["step"]), {k: v.get("traffic_over_algorithmic") for k, v in kernels.items() if "traffic_over_algorithmic" in v})


if __name__ == "__main__":
    main()
