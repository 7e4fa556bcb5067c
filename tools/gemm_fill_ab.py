"""A/B of GEMM tile geometries on the config-5 shapes that fill the chip poorly (M = 4096, N = 1280: 320
128x128 tiles on 256 CUs): production pick vs the diagnostic 128x160 tiles (geometry 1601: 4 waves of
64x80; 1602: 8 waves of 32x80; 256 tiles = one per CU), forward direction (k-major operands). Outputs
compared bitwise, then per-call time (interleaved rounds, medians).

  VPT_DIAG=1 python tools/gemm_fill_ab.py [--rounds 5]
"""
import os
os.environ.setdefault("VPT_DIAG", "1")

import argparse
import json
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--geos", default="0,128,1601,1602")
    args = ap.parse_args()
    geos = [int(v) for v in args.geos.split(",")]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * s).bfloat16()

    shapes = {"M4096_N1280_K1280": (4096, 1280, 1280), "M4096_N1280_K5120": (4096, 1280, 5120),
              "M924_N1280_K2048": (924, 1280, 2048), "M16384_N640_K640": (16384, 640, 640)}
    cases = {}
    for name, (M, N, K) in shapes.items():
        x, w, b = rnd(M, K), rnd(N, K, s=0.05), rnd(N, s=0.05)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        cases[name] = (2.0 * M * N * K, lambda x=x, w=w, b=b, y=y: ops.linear(x, w, b, out=y), y)
    same, res = {}, {}
    for name, (fl, fn, out) in cases.items():
        ref = None
        for geo in geos:
            ops.lib.vpt_gemm_set_geometry(geo)
            out.zero_()
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            else:
                same[f"{name}@{geo}"] = bool(torch.equal(ref, out))
    for _ in range(args.rounds):
        for name, (fl, fn, out) in cases.items():
            for geo in geos:
                ops.lib.vpt_gemm_set_geometry(geo)
                res.setdefault(f"{name}@{geo}", []).append(timeit(fn) * 1e3)
    ops.lib.vpt_gemm_set_geometry(0)
    out = {"bitwise_equal": same, "us": {}, "tflops": {}}
    for k, v in res.items():
        us = sorted(v)[len(v) // 2]
        out["us"][k] = round(us, 2)
        out["tflops"][k] = round(cases[k.split("@")[0]][0] / (us * 1e-6) / 1e12, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
