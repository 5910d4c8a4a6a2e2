"""Kernel timeline of one decode step from a rocprofv3 kernel trace:
python tools/step_timeline.py <kernel_trace.csv> <anchor kernel substring> [step index from the end]
Groups dispatches into steps by the anchor kernel's launches (gaps), prints
each kernel of the chosen step (stream, start / end relative to the step, us)
and the per-stream busy time."""
import csv
import sys


def main():
    path, anchor = sys.argv[1], sys.argv[2]
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    an = [r for r in rows if anchor in r["Kernel_Name"]]
    # steps: clusters of anchor launches separated by > 1 ms of no anchor
    steps, cur = [], [an[0]]
    for r in an[1:]:
        if r["s"] - cur[-1]["e"] > 1_000_000:
            steps.append(cur)
            cur = [r]
        else:
            cur.append(r)
    steps.append(cur)
    st = steps[-back]
    t0 = min(r["s"] for r in st)
    t1 = max(r["e"] for r in st)
    # widen to every kernel overlapping [t0 - 0.5 ms, t1 + 0.5 ms] that touches the step's span
    win = [r for r in rows if r["e"] > t0 - 200_000 and r["s"] < t1 + 200_000]
    t0 = min(r["s"] for r in win)
    busy = {}
    for r in win:
        q = r["Queue_Id"]
        busy[q] = busy.get(q, 0) + r["e"] - r["s"]
        print(f"q{q:>3} {(r['s'] - t0) / 1e3:9.1f} {(r['e'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f}  {r['Kernel_Name'][:70]}")
    print("span us", (max(r["e"] for r in win) - t0) / 1e3, "busy per queue us", {k: v / 1e3 for k, v in busy.items()})


if __name__ == "__main__":
    main()
