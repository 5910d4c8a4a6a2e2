"""HBM traffic of the decode kernel from rocprofv3 PMC counters.

Collected in two separate --pmc passes (FETCH_SIZE and WRITE_SIZE do not
fit one TCC pass), as MI355X_MICROARCH.md §HBM prescribes, and corrected
for gfx950: FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane)
coalesced streaming read -- the page staging here is 16 B/lane LDS-DMA,
so fetch bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16 B/lane
streaming stores (write bytes = WRITE_SIZE x 1024).

usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> <workload> <algorithmic_bytes>
Updates profiles/pmc_traffic.json[workload] with per-launch bytes.
"""
import csv
import json
import os
import sys

KERNEL = "k_decode_staged"


def per_dispatch(path, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fetch_csv, write_csv, workload, alg = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    f = per_dispatch(fetch_csv, "FETCH_SIZE")
    w = per_dispatch(write_csv, "WRITE_SIZE")
    assert f and w, "no decode dispatches found"
    # skip the first (cold) dispatch of each pass
    f_avg = sum(f[1:] or f) / len(f[1:] or f)
    w_avg = sum(w[1:] or w) / len(w[1:] or w)
    fetch_b = 2.0 * f_avg * 1024
    write_b = w_avg * 1024
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles", "pmc_traffic.json")
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[workload] = {
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "fetch_bytes_per_launch": int(fetch_b),
        "write_bytes_per_launch": int(write_b),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((fetch_b + write_b) / alg, 4),
        "dispatches": [len(f), len(w)],
        "correction": "fetch = 2 x FETCH_SIZE x 1KiB (gfx950 16 B/lane read undercount), write = WRITE_SIZE x 1KiB",
    }
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(data[workload]))


if __name__ == "__main__":
    main()
