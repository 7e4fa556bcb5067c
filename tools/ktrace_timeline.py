"""Timeline view of a multi-stream rocprofv3 --kernel-trace run of bench.py: per step, the time with no kernel running
(dispatch gaps / waits), the time with exactly one and with two or more kernels in flight, and the largest idle gaps
with the kernels on either side.
    python tools/ktrace_timeline.py gpurun_out/<tag>/ktrace_side"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ktrace_summary import family  # noqa: E402


def main():
    d = sys.argv[1]
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "radam" in r["Kernel_Name"]]
    seg = rows[marks[0] + 1:marks[-1] + 1]
    steps = len(marks) - 1
    t0 = int(rows[marks[0]]["End_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    ev = []
    for r in seg:
        ev.append((int(r["Start_Timestamp"]), 1, r))
        ev.append((int(r["End_Timestamp"]), -1, r))
    ev.sort(key=lambda e: (e[0], e[1]))
    cur, last, last_end = 0, t0, rows[marks[0]]
    acc = {0: 0.0, 1: 0.0, 2: 0.0}
    gaps = []
    for t, dlt, r in ev:
        span = t - last
        acc[min(cur, 2)] += span
        if cur == 0 and span > 0:
            gaps.append((span, family(last_end["Kernel_Name"]), family(r["Kernel_Name"])))
        cur += dlt
        if dlt < 0:
            last_end = r
        last = t
    wall = (t1 - t0) / steps / 1e6
    print(f"{steps} steps: wall {wall:.3f} ms/step; no kernel {acc[0] / steps / 1e6:.3f} ms, one {acc[1] / steps / 1e6:.3f} ms, "
          f"two or more {acc[2] / steps / 1e6:.3f} ms per step; {len(gaps) / steps:.0f} idle gaps per step")
    gaps.sort(reverse=True)
    agg = {}
    for g, a, b in gaps:
        k = (a, b)
        n, s = agg.get(k, (0, 0.0))
        agg[k] = (n + 1, s + g)
    print("idle time by (kernel before, kernel after), us per step:")
    for (a, b), (n, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {s / steps / 1e3:8.1f} us  {n / steps:5.1f}x  {a} -> {b}")


if __name__ == "__main__":
    main()
