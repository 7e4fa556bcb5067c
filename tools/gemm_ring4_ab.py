"""A/B of the 4-wave ring GEMM (diag geometry 2569, csrc/diag/gemm_ring4.inc) against the production 8-wave
ring (256) at the JiT-B/16 1024^2 B=8 shapes: every output compared bitwise (same MFMA sequence per output
element, so the results must be identical), then per-call time, interleaved rounds, medians.

  VPT_DIAG=1 python tools/gemm_ring4_ab.py [--rounds 5] [--M 33360]
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


def timeit(fn, iters=20):
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
    ap.add_argument("--M", type=int, default=8 * 4170)
    ap.add_argument("--geos", default="256,2569")
    ap.add_argument("--only", default="", help="substring filter on case names (ablation geometries: fwd only)")
    args = ap.parse_args()
    geos = [int(v) for v in args.geos.split(",")]
    dev = "cuda"
    M, D, F = args.M, 768, 2048
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, device=dev, generator=g) * s).bfloat16()

    ws = torch.empty(8 * 4096 * 4096, dtype=torch.float32, device=dev)
    cases = {}
    for name, (N, K) in {"qkv": (3 * D, D), "o": (D, D), "w12": (2 * F, D), "w3": (D, F)}.items():
        x, w, b, dy = rnd(M, K), rnd(N, K, s=0.05), rnd(N, s=0.05), rnd(M, N)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        dw = torch.empty(N, K, dtype=torch.float32, device=dev)
        sp = ops.wgrad_splits(N, K, M)
        fl = 2.0 * M * N * K
        cases[f"{name}.fwd"] = (fl, lambda x=x, w=w, b=b, y=y: ops.linear(x, w, b, out=y), y)
        if name in ("o", "w3"):
            r = rnd(M, N)
            cases[f"{name}.fwd_resid"] = (fl, lambda x=x, w=w, b=b, y=y, r=r: ops.linear(x, w, b, resid=r, out=y), y)
        cases[f"{name}.dgrad"] = (fl, lambda dy=dy, w=w, dx=dx: ops.linear_dgrad(dy, w, out=dx), dx)
        cases[f"{name}.wgrad_s{sp}"] = (fl, lambda dy=dy, x=x, dw=dw, sp=sp: ops.linear_wgrad(dy, x, dw, splits=sp,
                                                                                                workspace=ws), dw)
    dy, w3 = rnd(M, D), rnd(D, F, s=0.05)
    x12 = rnd(M, 2 * F)
    dx12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=dev)
    dh = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
    cases["swiglu_bwd.fused"] = (2.0 * M * F * D, lambda: ops.linear_dgrad_swiglu(dy, w3, x12, dx12, workspace=dh),
                                 dx12)

    if args.only:
        cases = {k: v for k, v in cases.items() if args.only in k}
    same = {}
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
        ops.lib.vpt_gemm_set_geometry(0)
    res = {}
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
    tot = {geo: sum(out["us"][f"{n}@{geo}"] for n in cases) for geo in geos}
    out["sum_us"] = {str(k): round(v, 1) for k, v in tot.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
