"""In-process A/B of the attention backward's two launch forms at the C3 and C2 shapes: one block per dK/dV / dQ item
(vpt_attn_bwd) vs resident blocks pulling the same items from per-XCD work queues (vpt_attn_bwd_q). Outputs compared
bitwise; per-launch medians over interleaved rounds (HIP events on the launching stream).

  python tools/attn_queue_ab.py [--rounds 8] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vpt import ops  # noqa: E402

# (B, n rows, always-valid keys): C3 = 8 x (4096 patches + 10 tokens + 64 context rows), C2 = 16 x (1024 + 10 + 64)
SHAPES = {"c3": (8, 4170, 4106), "c2": (16, 1098, 1034)}


def case(dev, B, n, nd, H=12):
    D = 64 * H
    M = B * n
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(M, 3 * D, device=dev, generator=g).bfloat16()
    wq = (1 + 0.1 * torch.randn(64, device=dev, generator=g)).bfloat16()
    wk = (1 + 0.1 * torch.randn(64, device=dev, generator=g)).bfloat16()
    ang = torch.rand(n, 32, device=dev, generator=g) * 6
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    qk = ops.qknorm_rope_fwd(qkv, wq, wk, cos, sin, n, q_scale=ops.attn_q_scale(0.125))
    kb = torch.zeros(B, n, device=dev)
    kb[:, nd + 30:] = float("-inf")
    o = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, n, device=dev)
    do = torch.randn(M, D, device=dev, generator=g).bfloat16()
    dqkv = torch.zeros(M, 3 * D, dtype=torch.bfloat16, device=dev)
    dqk = torch.zeros(M, 2 * D, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B, H, n, device=dev)
    q4, k4, v4 = ops._t4(qk, B, n, H, 0), ops._t4(qk, B, n, H, D), ops._t4(qkv, B, n, H, 2 * D)
    o4, do4 = ops._t4(o, B, n, H, 0), ops._t4(do, B, n, H, 0)
    ops.attn_fwd_qknorm(q4, k4, v4, o4, lse, kb, wq, wk, B, H, n, n, nd)

    def bwd(queue):
        ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                     ops._t4(dqkv, B, n, H, 2 * D), B, H, n, n, nd, queue=queue)
    return bwd, (dqk, dqkv), (qk, qkv, o, do, lse, kb)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="c3,c2")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    for name in args.shapes.split(","):
        B, n, nd = SHAPES[name]
        bwd, res, keep = case(dev, B, n, nd)
        got = {}
        for qv in (False, True, True):
            bwd(qv)
            torch.cuda.synchronize()
            cur = [t.clone() for t in res]
            if qv in got:
                assert all(torch.equal(a, b) for a, b in zip(got[qv], cur)), "queue run not reproducible"
            got[qv] = cur
        equal = all(torch.equal(a, b) for a, b in zip(got[False], got[True]))
        tm = {"grid": [], "queue": []}
        st = torch.cuda.current_stream()
        for r in range(args.rounds):
            for qv in ((False, True) if r % 2 == 0 else (True, False)):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
                bwd(qv)
                ev[0].record(st)
                for i in range(args.iters):
                    bwd(qv)
                    ev[i + 1].record(st)
                torch.cuda.synchronize()
                tm["queue" if qv else "grid"].append(statistics.median(ev[i].elapsed_time(ev[i + 1])
                                                                       for i in range(args.iters)))
        med = {k: round(statistics.median(v), 4) for k, v in tm.items()}
        fl = 8.0 * B * 12 * n * n * 64
        out[name] = {"bitwise_equal": equal, "median_ms": med, "ratio_queue_to_grid": round(med["queue"] / med["grid"], 4),
                     "tflops": {k: round(fl / (v * 1e-3) / 1e12, 1) for k, v in med.items()},
                     "rounds_ms": {k: [round(x, 4) for x in v] for k, v in tm.items()}}
        print(name, json.dumps(out[name]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
