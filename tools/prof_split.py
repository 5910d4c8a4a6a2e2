"""Per-workload kernel durations from a rocprofv3 kernel trace of bench.py.

bench.py launches the decode kernel for the C2 headline mix, the harder C2
mix and the b12 variant (warmup + steps each, in that order); all use
k_decode_staged<4,false>, so the --stats summary averages them.  This splits the trace by dispatch
order and reports the timed launches of each workload.

usage: python tools/prof_split.py <kernel_trace.csv> <warmup> <steps> [out.json]
"""
import csv
import json
import sys


def main():
    path, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = [r for r in csv.DictReader(open(path)) if "k_decode_staged" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    per = warm + steps
    out = {}
    for i, name in enumerate(["c2_int32_adaptive_bitpack_dict", "c2_hard_mix", "bitpack_b12"]):
        seg = dur[i * per:(i + 1) * per][warm:]
        if seg:
            out[name] = {"kernel": rows[0]["Kernel_Name"], "timed_dispatches": len(seg),
                         "avg_us": round(sum(seg) / len(seg), 2), "min_us": round(min(seg), 2),
                         "max_us": round(max(seg), 2)}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(s + "\n")


if __name__ == "__main__":
    main()
