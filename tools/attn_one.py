"""Runs the production attention forward + backward at the bench shape (JiT-B/16, B=8, 1024^2: n = 4170,
12 heads, 64 context keys with a ragged valid length) `--iters` times; a driver for rocprofv3 counter passes.

  python tools/attn_one.py [--iters 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--time", action="store_true", help="print median ms per forward / backward launch (JSON)")
    ap.add_argument("--rows64", type=int, default=None,
                    help="diagnostic library (VPT_DIAG=1): vpt_attn_set_rows64 mask; 8 = the production dK/dV and dQ "
                         "bodies as two separate launches (per-kind kernel times under rocprofv3)")
    args = ap.parse_args()
    if args.rows64 is not None:
        ops.lib.vpt_attn_set_rows64(args.rows64)
    dev = "cuda"
    B, H, n = 8, 12, 4170
    rows, D = n, 768
    n_dense = n - 64
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * rows, 3 * D, device=dev, generator=g).bfloat16()
    qkv[:, :D] = (qkv[:, :D].float() * ops.attn_q_scale(0.125)).bfloat16()
    kb = torch.zeros(B, rows, device=dev)
    for b in range(B):
        kb[b, n_dense + 8 + 7 * b:] = float("-inf")
    o = torch.empty(B * rows, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, rows, device=dev)
    delta = torch.empty_like(lse)
    do = torch.randn(B * rows, D, device=dev, generator=g).bfloat16()
    dqk = torch.empty(B * rows, 2 * D, dtype=torch.bfloat16, device=dev)
    dv = torch.empty(B * rows, D, dtype=torch.bfloat16, device=dev)
    q4, k4, v4 = (ops._t4(qkv, B, rows, H, c) for c in (0, D, 2 * D))
    o4 = ops._t4(o, B, rows, H)
    fwd = lambda: ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense)  # noqa: E731
    bwd = lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb,  # noqa: E731
                               ops._t4(dqk, B, rows, H, 0), ops._t4(dqk, B, rows, H, D), ops._t4(dv, B, rows, H),
                               B, H, rows, n, n_dense)
    if not args.time:
        for _ in range(args.iters):
            fwd()
            bwd()
        torch.cuda.synchronize()
        print("ok")
        return
    import json
    import statistics
    res = {"fwd": [], "bwd": []}
    for _ in range(args.iters):
        for k, fn in (("fwd", fwd), ("bwd", bwd)):
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[k].append(s.elapsed_time(e) / 10)
    print(json.dumps({k: round(statistics.median(v), 4) for k, v in res.items()}))


if __name__ == "__main__":
    main()
