"""The 256x128 two-blocks-per-CU ring (gemm_r2.hip) against the 256x256 ring at the JiT-B/16 C3 shapes (M = B * rows,
B = 8), every launch kind of the step: forward with the fused QK-norm + RoPE epilogue, forwards with a residual, the
fused SwiGLU forward and backward, input gradients and weight gradients (split-K, fused bias gradient). Outputs must be
bitwise equal (same per-wave tile, K order and epilogue); times are medians of interleaved rounds (HIP events).
Diagnostic library (vpt_gemm_set_r2).

  python tools/r2_ab.py [--M 32848] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    s = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    s[0].record()
    for i in range(iters):
        fn()
        s[i + 1].record()
    torch.cuda.synchronize()
    return statistics.median(s[i].elapsed_time(s[i + 1]) for i in range(iters)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8 * 4106)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--mask", type=int, default=31)
    ap.add_argument("--lib", default=None, help="a diagnostic variant build lib/var/libvpt_hip_<name>.so")
    ap.add_argument("--only", default=None, help="cases whose name contains this")
    ap.add_argument("--stagger", type=int, default=0, help="R2 start stagger of the second blocks (10-ns ticks)")
    args = ap.parse_args()
    if args.lib:
        from vpt._build import PKG_ROOT
        _lib.use_library(PKG_ROOT / "lib" / "var" / f"libvpt_hip_{args.lib}.so", diag=True)
    else:
        _lib.use_diag()
    dev = "cuda"
    M, D, F = args.M, 768, 2048
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).bfloat16()  # noqa: E731
    x, h = rnd(M, D), rnd(M, F)
    wqkv, bqkv = rnd(3 * D, D, sc=0.03), rnd(3 * D, sc=0.1)
    wo, bo, w3, b3 = rnd(D, D, sc=0.03), rnd(D, sc=0.1), rnd(D, F, sc=0.03), rnd(D, sc=0.1)
    w12, b12 = rnd(2 * F, D, sc=0.03), rnd(2 * F, sc=0.1)
    wq, wk = rnd(64, sc=0.1) + 1, rnd(64, sc=0.1) + 1
    cos, sin = torch.rand(4106, 32, device=dev), torch.rand(4106, 32, device=dev)
    resid, dy, x12 = rnd(M, D), rnd(M, D), rnd(M, 2 * F)
    dqkv, dx12 = rnd(M, 3 * D), rnd(M, 2 * F)
    outs = {k: torch.empty(*s, dtype=torch.bfloat16, device=dev) for k, s in
            (("qkv", (M, 3 * D)), ("qk", (M, 2 * D)), ("o", (M, D)), ("w3", (M, D)), ("x12", (M, 2 * F)), ("h", (M, F)),
             ("dx12", (M, 2 * F)), ("dxo", (M, D)), ("dxqkv", (M, D)), ("dx12b", (M, D)))}
    wg = {k: torch.empty(n, kk, dtype=torch.float32, device=dev) for k, n, kk in
          (("gqkv", 3 * D, D), ("go", D, D), ("g12", 2 * F, D), ("g3", D, F))}
    gb = {k: torch.empty(n, dtype=torch.float32, device=dev) for k, n in (("gqkv", 3 * D), ("go", D), ("g12", 2 * F),
                                                                           ("g3", D))}
    cases = {
        "fwd+qkn N2304 K768": (lambda: ops.linear_qknorm_rope(x, wqkv, bqkv, outs["qkv"], outs["qk"], wq, wk, cos, sin,
                                                               4106, q_scale=0.18), ("qkv", "qk"), 2 * M * 3 * D * D),
        "fwd+resid N768 K768": (lambda: ops.linear(x, wo, bo, resid=resid, out=outs["o"]), ("o",), 2 * M * D * D),
        "fwd+resid N768 K2048": (lambda: ops.linear(h, w3, b3, resid=resid, out=outs["w3"]), ("w3",), 2 * M * D * F),
        "swiglu_fwd N4096 K768": (lambda: ops.linear_swiglu(x, w12, b12, outs["x12"], outs["h"]), ("x12", "h"),
                                  2 * M * 2 * F * D),
        "swiglu_dgrad N2048 K768": (lambda: ops.linear_dgrad_swiglu(dy, w3, x12, outs["dx12"]), ("dx12",),
                                    2 * M * F * D),
        "dgrad N768 K768": (lambda: ops.linear_dgrad(dy, wo, out=outs["dxo"]), ("dxo",), 2 * M * D * D),
        "dgrad N768 K2304": (lambda: ops.linear_dgrad(dqkv, wqkv, out=outs["dxqkv"]), ("dxqkv",), 2 * M * D * 3 * D),
        "dgrad N768 K4096": (lambda: ops.linear_dgrad(dx12, w12, out=outs["dx12b"]), ("dx12b",), 2 * M * D * 2 * F),
    }
    for name, dyt, xt, key, N, K in (("wgrad N2304 K768", dqkv, x, "gqkv", 3 * D, D),
                                        ("wgrad N768 K768", dy, x, "go", D, D),
                                        ("wgrad N4096 K768", dx12, x, "g12", 2 * F, D),
                                        ("wgrad N768 K2048", dy, h, "g3", D, F)):
        sp = ops.wgrad_splits(N, K, M)
        cases[f"{name} s{sp}"] = ((lambda dyt=dyt, xt=xt, key=key, sp=sp: ops.linear_wgrad(
            dyt, xt, wg[key], splits=sp, bias_out=gb[key])), (key, "b:" + key), 2 * M * N * K)

    def grab(names):
        return [(wg[n] if n in wg else gb[n[2:]] if n.startswith("b:") else outs[n]).clone() for n in names]

    res = {}
    for name, (fn, names, fl) in cases.items():
        if args.only and args.only not in name:
            continue
        got = {}
        for m in (0, args.mask):
            _lib.lib.vpt_gemm_set_r2(m)
            _lib.lib.vpt_gemm_set_stagger(args.stagger if m else 0)  # the stagger for the R2 side only
            fn()
            torch.cuda.synchronize()
            got[m] = grab(names)
        eq = all(torch.equal(a, b) for a, b in zip(got[0], got[args.mask]))
        t = {0: [], args.mask: []}
        for r in range(args.rounds):
            for m in ((0, args.mask) if r % 2 == 0 else (args.mask, 0)):
                _lib.lib.vpt_gemm_set_r2(m)
                _lib.lib.vpt_gemm_set_stagger(args.stagger if m else 0)
                t[m].append(timeit(fn))
        ring, r2 = statistics.median(t[0]), statistics.median(t[args.mask])
        res[name] = {"bitwise_equal": eq, "ring_us": round(ring, 1), "r2_us": round(r2, 1),
                     "r2_vs_ring": round(r2 / ring, 4), "ring_tflops": round(fl / ring / 1e6, 1),
                     "r2_tflops": round(fl / r2 / 1e6, 1)}
        print(name, json.dumps(res[name]), flush=True)
    _lib.lib.vpt_gemm_set_r2(8)  # production
    _lib.lib.vpt_gemm_set_stagger(0)
    print(json.dumps({"M": M, "lib": args.lib, "stagger": args.stagger, "cases": res}))


if __name__ == "__main__":
    main()
