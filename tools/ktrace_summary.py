"""Per-step kernel-time breakdown of a rocprofv3 --kernel-trace run of bench.py (one line per kernel family).
    python tools/ktrace_summary.py gpurun_out/<tag>/ktrace [steps]"""
import csv
import os
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    n = name.split("(anonymous namespace)::", 1)[1] if "(anonymous namespace)::" in name else name
    if n.startswith("gemm_ring_kernel"):
        m = re.match(r"gemm_ring_kernel<(\w+), (\w+), \w+, (\d+), \w+, \w+, \w+, (\d+), (\d+)", n)
        return "gemm_ring<AK=%s,BK=%s,SW=%s,EPI=%s>" % (m.group(1)[0], m.group(2)[0], m.group(4), m.group(5)) if m else n[:40]
    if "at::native" in name:
        return "torch:" + (re.search(r"(\w+Functor|\w+_kernel\w*)", name) or [None, name[:30]])[1]
    return re.split(r"[<(]", n)[0]


def main():
    d = sys.argv[1]
    rows = list(csv.DictReader(open(os.path.join(d, "p_kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "radam" in r["Kernel_Name"]]
    steps = len(marks) - 1
    seg = rows[marks[0] + 1:marks[-1] + 1]
    t = defaultdict(float)
    c = defaultdict(int)
    for r in seg:
        f = family(r["Kernel_Name"])
        t[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c[f] += 1
    wall = (int(seg[-1]["End_Timestamp"]) - int(rows[marks[0]]["End_Timestamp"])) / 1e3 / steps
    tot = sum(t.values()) / steps
    print(f"{steps} steps: wall {wall / 1e3:.3f} ms/step, kernel sum {tot / 1e3:.3f} ms/step")
    for f, v in sorted(t.items(), key=lambda kv: -kv[1]):
        print(f"{v / steps / 1e3:8.3f} ms {c[f] / steps:6.1f}/step {v / c[f]:8.1f} us  {f}")


if __name__ == "__main__":
    main()
