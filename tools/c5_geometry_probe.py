"""Tile-geometry probe of config 5's half-empty base+LoRA GEMMs (M ~ 4100 tokens x N 1280 x K 1280, forward and input
gradient, r = 16 extension, bias + residual on the forward): the production 128x128 kernel against the 256x256 ring
and the 256x128 two-blocks-per-CU ring (R2, diagnostic library switch vpt_gemm_set_r2), the outputs compared bitwise
between the two ring geometries. Interleaved rounds, medians of HIP-event times.

  python tools/c5_geometry_probe.py [--rounds 5]
  python tools/c5_geometry_probe.py --plan [--rounds 5]   (production library: 128 / 1281 / 256 ring / ops' plan, more
                                                           shapes of the C5 step)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402


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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--plan", action="store_true")
    args = ap.parse_args()
    if args.plan:
        return plan_probe(args.rounds)
    _lib.use_diag()
    dev = "cuda"
    res = {}
    for M, Nw, Kw in ((4224, 1280, 1280), (4032, 1280, 1280), (4224, 1280, 5120), (4224, 1280, 3840)):
        for fwd in (True, False):
            N, K = (Nw, Kw) if fwd else (Kw, Nw)
            if not fwd and Kw != 1280:
                continue
            W = (torch.randn(Nw, Kw, device=dev) * 0.03).to(torch.bfloat16)
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            a2 = (torch.randn(M, 16, device=dev) * 0.5).to(torch.bfloat16)
            b2 = ((torch.randn(N, 16, device=dev) if fwd else torch.randn(16, N, device=dev)) * 0.1).to(torch.bfloat16)
            bias = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16) if fwd else None
            resid = torch.randn(M, N, device=dev).to(torch.bfloat16) if fwd else None
            outs = {k: torch.empty(M, N, dtype=torch.bfloat16, device=dev) for k in ("t128", "ring", "r2")}
            kinds = {"t128": (128, 8), "ring": (256, 8), "r2": (256, 9)}

            def run(k):
                geo, mask = kinds[k]
                _lib.lib.vpt_gemm_set_r2(mask)
                ops.gemm_lora(a, W, fwd, a2, b2, M, N, K, outs[k], bias=bias, resid=resid, geometry=geo, splits=1)
            t = {k: [] for k in kinds}
            for _ in range(args.rounds):
                for k in kinds:
                    t[k].append(timeit(lambda: run(k)))
            _lib.lib.vpt_gemm_set_r2(8)
            med = {k: round(sorted(v)[len(v) // 2], 1) for k, v in t.items()}
            key = f"{'fwd' if fwd else 'dgrad'} M{M} N{N} K{K}"
            res[key] = {"us": med, "ring_eq_r2": bool(torch.equal(outs["ring"], outs["r2"])),
                        "t128_vs_ring_maxdiff": (outs["t128"].float() - outs["ring"].float()).abs().max().item()}
            print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


def plan_probe(rounds):
    dev = "cuda"
    res = {}
    shapes = [(4224, 1280, 1280, True), (4224, 1280, 1280, False), (4224, 5120, 1280, False), (4224, 1280, 5120, True),
              (4224, 1280, 3840, False), (16896, 640, 640, True), (16896, 640, 640, False), (16896, 640, 2560, True),
              (16896, 2560, 640, False), (16896, 640, 1920, False), (16896, 1920, 640, True), (16896, 5120, 640, True)]
    for M, N, K, fwd in shapes:
        W = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16) if fwd else \
            (torch.randn(K, N, device=dev) * 0.03).to(torch.bfloat16)
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        a2 = (torch.randn(M, 16, device=dev) * 0.5).to(torch.bfloat16)
        b2 = ((torch.randn(N, 16, device=dev) if fwd else torch.randn(16, N, device=dev)) * 0.1).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        plan = ops.lora_gemm_plan(M, N, K)
        kinds = {"t128": (128, 1), "r2_128": (1281, 1), "ring": (256, 1), "plan": plan}
        t = {k: [] for k in kinds}
        for _ in range(rounds):
            for k, (geo, sp) in kinds.items():
                t[k].append(timeit(lambda: ops.gemm_lora(a, W, fwd, a2, b2, M, N, K, out, geometry=geo, splits=sp)))
        key = f"{'fwd' if fwd else 'dgrad'} M{M} N{N} K{K}"
        res[key] = {"plan": list(plan), "us": {k: round(sorted(v)[len(v) // 2], 1) for k, v in t.items()}}
        print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
