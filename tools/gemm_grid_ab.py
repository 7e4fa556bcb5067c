"""Persistent ring grid (one block per CU walking items) vs one block per item, same process, interleaved rounds,
at the C3 bench shapes (M = 8 x 4170): every ring GEMM of a JiT-B/16 block (forward, fused SwiGLU forward / backward,
input and weight gradients). Diagnostic library (vpt_gemm_set_ring_grid). Prints per-shape medians (us) and the sum.

  python tools/gemm_grid_ab.py [--rounds 5]
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
    _lib.use_diag()
    dev = "cuda"
    M, D, F = args.M, 768, 2048
    r = lambda *s: torch.randn(*s, device=dev).bfloat16()  # noqa: E731
    w = lambda *s: (torch.randn(*s, device=dev) * 0.05).bfloat16()  # noqa: E731
    x, xo, h = r(M, D), r(M, D), r(M, F)
    wqkv, bqkv, wo, bo, w12, b12, w3, b3 = w(3 * D, D), w(3 * D), w(D, D), w(D), w(2 * F, D), w(2 * F), w(D, F), w(D)
    yqkv, y, x12, hh = (torch.empty(M, n, dtype=torch.bfloat16, device=dev) for n in (3 * D, D, 2 * F, F))
    dqkv, dy, dx12 = r(M, 3 * D), r(M, D), r(M, 2 * F)
    dx = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    dxf = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
    ws = torch.empty(64 * 4096 * 2048, dtype=torch.float32, device=dev)
    dws = {n: torch.empty(*s, dtype=torch.float32, device=dev) for n, s in
           (("qkv", (3 * D, D)), ("o", (D, D)), ("w12", (2 * F, D)), ("w3", (D, F)))}
    dbs = {n: torch.empty(s, dtype=torch.float32, device=dev) for n, s in (("qkv", 3 * D), ("o", D), ("w12", 2 * F),
                                                                           ("w3", D))}

    def wg(dyt, xin, n):
        N, K = dyt.shape[1], xin.shape[1]
        ops.linear_wgrad(dyt, xin, dws[n], splits=ops.wgrad_splits(N, K, M), workspace=ws, bias_out=dbs[n])

    calls = {
        "qkv_fwd": lambda: ops.linear(x, wqkv, bqkv, out=yqkv),
        "o_fwd_resid": lambda: ops.linear(xo, wo, bo, resid=x, out=y),
        "swiglu_fwd": lambda: ops.linear_swiglu(x, w12, b12, x12, hh),
        "w3_fwd_resid": lambda: ops.linear(h, w3, b3, resid=x, out=y),
        "swiglu_dgrad": lambda: ops.linear_dgrad_swiglu(dy, w3, x12, dx12, workspace=dxf),
        "w12_dgrad": lambda: ops.linear_dgrad(dx12, w12, out=dx),
        "o_dgrad": lambda: ops.linear_dgrad(dy, wo, out=dx),
        "qkv_dgrad": lambda: ops.linear_dgrad(dqkv, wqkv, out=dx),
        "w3_wgrad": lambda: wg(dy, h, "w3"),
        "w12_wgrad": lambda: wg(dx12, x, "w12"),
        "o_wgrad": lambda: wg(dy, xo, "o"),
        "qkv_wgrad": lambda: wg(dqkv, x, "qkv"),
    }
    res = {(k, m): [] for k in calls for m in (0, 1)}
    for rd in range(args.rounds):
        for m in ((0, 1) if rd % 2 == 0 else (1, 0)):
            _lib.lib.vpt_gemm_set_ring_grid(0 if m else 256)
            for k, fn in calls.items():
                res[(k, m)].append(timeit(fn))
    _lib.lib.vpt_gemm_set_ring_grid(0)
    out = {k: {"persistent": round(statistics.median(res[(k, 0)]), 1), "per_item": round(statistics.median(res[(k, 1)]), 1)}
           for k in calls}
    tot = {m: round(sum(v[m] for v in out.values()), 1) for m in ("persistent", "per_item")}
    print(json.dumps({"M": M, "us": out, "sum_us": tot}, indent=1))


if __name__ == "__main__":
    main()
