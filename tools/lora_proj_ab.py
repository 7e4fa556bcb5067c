"""In-process A/B of vpt_lora_proj between builds of the library (lib/var/libvpt_hip_<name>.so; "base" =
lib/libvpt_hip.so) at config 5's shapes, both W layouts; HIP-event medians per launch, outputs compared bitwise.

  python tools/lora_proj_ab.py --variants base,lpc
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402
from vpt._build import LIB, PKG_ROOT  # noqa: E402


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    libs = {v: _lib.load_library(LIB if v == "base" else PKG_ROOT / "lib" / "var" / f"libvpt_hip_{v}.so")
            for v in args.variants.split(",")}
    dev = "cuda"
    res = {}
    for M, K in ((4224, 1280), (4100, 1280), (16896, 640), (928, 2048)):
        x = torch.randn(M, K, device=dev).bfloat16()
        down = (torch.randn(16, K, device=dev) * 0.05).bfloat16()
        up = (torch.randn(K, 16, device=dev) * 0.05).bfloat16()
        cases = {"down": lambda o: ops.lora_proj(x, down, True, o, alpha=0.5),
                 "up": lambda o: ops.lora_proj(x, up, False, o, alpha=0.5)}
        t = {(v, c): [] for v in libs for c in cases}
        bufs = {c: torch.empty(M, 16, dtype=torch.bfloat16, device=dev) for c in cases}
        for _ in range(args.rounds):
            for v, lb in libs.items():
                _lib.use_library(lb)
                for c, fn in cases.items():
                    t[(v, c)].append(timeit(lambda: fn(bufs[c])))
        outs = {}
        for v, lb in libs.items():
            _lib.use_library(lb)
            o = {c: torch.full((M, 16), float("nan"), dtype=torch.bfloat16, device=dev) for c in cases}
            for c, fn in cases.items():
                fn(o[c])
            torch.cuda.synchronize()
            outs[v] = o
        _lib.use_library(libs[next(iter(libs))])
        key = f"{M}x{K}"
        res[key] = {f"{v}:{c}": round(sorted(x_)[len(x_) // 2], 1) for (v, c), x_ in t.items()}
        first = outs[next(iter(outs))]
        res[key]["bitwise_equal"] = {v: all(torch.equal(o[c], first[c]) for c in cases) for v, o in outs.items()}
        print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
