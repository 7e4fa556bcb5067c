"""Per-shape timing of the production GEMM entry points at the JiT-B/16 1024^2 B=8 shapes (forward
epilogues, dgrads, wgrad with fused bias). Run it alternately with and without VPT_LIB_AB=<lib> for a
same-box A/B against another revision (tools/build_ab.py). Median us per call, one JSON line.

  python tools/gemm_ab.py [--rounds 5]
"""
import argparse
import json
import os
import statistics
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
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--M", type=int, default=8 * 4170)
    args = ap.parse_args()
    dev = "cuda"
    M, D, F = args.M, 768, 2048
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).bfloat16()  # noqa: E731
    x, xf, h = r(M, D), r(M, D), r(M, F)
    wqkv, bqkv, wo, bo = r(3 * D, D, sc=0.05), r(3 * D, sc=0.05), r(D, D, sc=0.05), r(D, sc=0.05)
    w12, b12, w3, b3 = r(2 * F, D, sc=0.05), r(2 * F, sc=0.05), r(D, F, sc=0.05), r(D, sc=0.05)
    qkv = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=dev)
    y = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    x12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=dev)
    hh = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
    dx12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=dev)
    dy, dqkv = r(M, D), r(M, 3 * D)
    dx = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    dw = torch.empty(3 * D, D, dtype=torch.float32, device=dev)
    db = torch.empty(3 * D, dtype=torch.float32, device=dev)
    sp = ops.wgrad_splits(3 * D, D, M)
    ws = torch.empty(max(1, ops.linear_wgrad_workspace_bytes(M, 3 * D, D, sp)), dtype=torch.uint8, device=dev)
    ops.linear_swiglu(x, w12, b12, x12, hh)
    cases = {
        "qkv_fwd": lambda: ops.linear(x, wqkv, bqkv, out=qkv),
        "o_fwd_resid": lambda: ops.linear(x, wo, bo, resid=xf, out=y),
        "w3_fwd_resid": lambda: ops.linear(h, w3, b3, resid=xf, out=y),
        "swiglu_fwd": lambda: ops.linear_swiglu(x, w12, b12, x12, hh),
        "swiglu_dgrad": lambda: ops.linear_dgrad_swiglu(dy, w3, x12, dx12),
        "qkv_dgrad": lambda: ops.linear_dgrad(dqkv, wqkv, out=dx),
        "qkv_wgrad_bias": lambda: ops.linear_wgrad(dqkv, x, out=dw, splits=sp, workspace=ws, bias_out=db),
    }
    res: dict = {}
    for _ in range(args.rounds):
        for name, fn in cases.items():
            res.setdefault(name, []).append(timeit(fn))
    out = {n: round(statistics.median(v), 2) for n, v in res.items()}
    out["_lib"] = os.environ.get("VPT_LIB_AB", "production")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
