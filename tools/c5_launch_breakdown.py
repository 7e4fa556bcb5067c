"""Per-entry-point time of one config-5 step: every C-ABI launch (vpt/_lib.call) bracketed with HIP events on the
launching stream during one SDXLFlowMatchQLoRA.step after warm-up, grouped by (entry point, small integer arguments --
the shape / layout flags; pointers and leading dims above 2^20 dropped). Prints JSON sorted by total time.

  python tools/c5_launch_breakdown.py [--top 40]
"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402
from vpt.sdxl_flow import SDXLFlowMatchQLoRA  # noqa: E402

SKIP = ("workspace_bytes", "last_error", "set_geometry")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    m = SDXLFlowMatchQLoRA(B=4, device="cuda", seed=0)
    lat, ctx, pooled, sizes = m.make_inputs(seed=1)
    for _ in range(2):
        m.step(lat, ctx, pooled, sizes)
    torch.cuda.synchronize()
    inner = ops.call
    rec = []

    def timed(name, *a):
        if any(s in name for s in SKIP):
            return inner(name, *a)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = inner(name, *a)
        e.record()
        key = tuple(v for v in a if isinstance(v, int) and 0 <= v < (1 << 20))
        rec.append((name, key, s, e))
        return rc

    ops.call = timed
    try:
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        m.step(lat, ctx, pooled, sizes)
        t1.record()
        torch.cuda.synchronize()
    finally:
        ops.call = inner
    tot = collections.defaultdict(lambda: [0, 0.0])
    per_name = collections.defaultdict(lambda: [0, 0.0])
    for name, key, s, e in rec:
        us = s.elapsed_time(e) * 1e3
        tot[(name, key)][0] += 1
        tot[(name, key)][1] += us
        per_name[name][0] += 1
        per_name[name][1] += us
    out = {"step_ms_with_events": round(t0.elapsed_time(t1), 3), "launches": len(rec),
           "sum_launch_ms": round(sum(v[1] for v in tot.values()) / 1e3, 3),
           "by_entry": {k: {"n": v[0], "ms": round(v[1] / 1e3, 3), "avg_us": round(v[1] / v[0], 1)}
                        for k, v in sorted(per_name.items(), key=lambda kv: -kv[1][1])},
           "by_shape": [{"entry": k[0], "ints": list(k[1]), "n": v[0], "ms": round(v[1] / 1e3, 3),
                         "avg_us": round(v[1] / v[0], 1)}
                        for k, v in sorted(tot.items(), key=lambda kv: -kv[1][1])[:args.top]]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
