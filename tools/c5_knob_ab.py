"""In-process A/B of config-5 module-level knobs: one SDXLFlowMatchQLoRA built once, then rounds of K timed steps
alternating the knob(s) on / off (vpt.sdxl globals read at call time, e.g. FOLD_Q_SCALE, FUSED_LN_LORA,
FUSED_LN_BWD_LORA; "ops.NAME" for a vpt.ops global, e.g. ops.LORA_SERIAL_SPLIT), so allocation, clocks and box are shared; medians of ms per step. The step and the optimizer
keep running across rounds (the values drift; the timing does not depend on them).

  python tools/c5_knob_ab.py FOLD_Q_SCALE [--rounds 6] [--steps 4] [--latent 96,176]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops, sdxl  # noqa: E402
from vpt.sdxl_flow import SDXLFlowMatchQLoRA  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knobs", help="comma-separated vpt.sdxl globals switched together")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--latent", default=None, help="H,W of the latent bucket (default: the model's, 128,128)")
    args = ap.parse_args()
    knobs = args.knobs.split(",")

    def where(k):  # "NAME" = vpt.sdxl.NAME, "ops.NAME" = vpt.ops.NAME
        return (ops, k[4:]) if k.startswith("ops.") else (sdxl, k)
    for k in knobs:
        mod, name = where(k)
        if not isinstance(getattr(mod, name), bool):
            raise SystemExit(f"{k}: not a boolean knob of {mod.__name__}")
    m = SDXLFlowMatchQLoRA(B=4, device="cuda", seed=0)
    lat, ctx, pooled, sizes = m.make_inputs(seed=1, latent=tuple(map(int, args.latent.split(","))) if args.latent else None)

    def setk(v):
        for k in knobs:
            setattr(*where(k), v)

    for v in (True, False):
        setk(v)
        for _ in range(2):
            m.step(lat, ctx, pooled, sizes)
    torch.cuda.synchronize()
    res = {"1": [], "0": []}
    for r in range(args.rounds):
        for v in ((True, False) if r % 2 == 0 else (False, True)):
            setk(v)
            m.step(lat, ctx, pooled, sizes)  # one untimed step after the switch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                m.step(lat, ctx, pooled, sizes)
            torch.cuda.synchronize()
            res["1" if v else "0"].append((time.perf_counter() - t0) / args.steps * 1e3)
        print(f"round {r}: on {res['1'][-1]:.3f} ms  off {res['0'][-1]:.3f} ms", flush=True)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(json.dumps({"knobs": knobs, "ms_per_step": {k: [round(x, 3) for x in v] for k, v in res.items()},
                      "median_ms": {k: round(v, 3) for k, v in med.items()},
                      "img_s_median": {k: round(4e3 / v, 3) for k, v in med.items()},
                      "gain": round(med["0"] / med["1"] - 1, 4)}))


if __name__ == "__main__":
    main()
