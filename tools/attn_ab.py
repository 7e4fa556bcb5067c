"""Same-process A/B of a diagnostic attention switch (diagnostic library) at the C3 shape (JiT-B/16, B=8, 1024^2: n = 4170
rows, 12 heads, QK-normed inputs): --setter vpt_attn_set_xcd_order (linear vs XCD-contiguous block order: a (batch,
head)'s blocks on one XCD), vpt_attn_set_fwd_order (the forward's S^T chain with its K fragments read first). Forward
(fixed reference) and backward launches timed with HIP events on the launching stream, values 0 and 1 interleaved over
rounds (medians); outputs checked bitwise equal between the two.

  python tools/attn_ab.py --setter vpt_attn_set_xcd_order [--rounds 8] [--iters 10]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--setter", default="vpt_attn_set_xcd_order")
    ap.add_argument("--value", type=int, default=1, help="the B value")
    ap.add_argument("--base", type=int, default=0, help="the A value")
    ap.add_argument("--shape", default="c3", choices=["c3", "c2"], help="c3: B=8, n=4170 (1024^2); c2: B=16, n=1098 (512^2)")
    args = ap.parse_args()
    _lib.use_diag()
    setter = getattr(_lib.lib, args.setter)
    dev = torch.device("cuda", 0)
    B, H, n, nd = (8, 12, 4170, 4106) if args.shape == "c3" else (16, 12, 1098, 1034)
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

    def fwd():
        ops.attn_fwd_qknorm(q4, k4, v4, o4, lse, kb, wq, wk, B, H, n, n, nd)

    def bwd():
        ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                     ops._t4(dqkv, B, n, H, 2 * D), B, H, n, n, nd)

    outs = {}
    for x in (0, 1):
        setter(args.value if x else args.base)
        fwd()
        bwd()
        torch.cuda.synchronize()
        outs[x] = (o.clone(), lse.clone(), dqk.clone(), dqkv.clone())
    equal = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    # variants that change the summation order (e.g. the 16x16x32 bodies): relative L2 of each output's difference
    D3 = {"o": (0, 0, D), "dq": (2, 0, D), "dk": (2, D, 2 * D), "dv": (3, 2 * D, 3 * D)}
    rel = {k: float((outs[1][i][:, a:b].float() - outs[0][i][:, a:b].float()).norm() / outs[0][i][:, a:b].float().norm())
           for k, (i, a, b) in D3.items()}
    st = torch.cuda.current_stream()
    res = {f"{k}{x}": [] for k in ("fwd", "bwd") for x in (0, 1)}
    for r in range(args.rounds):
        for x in ((0, 1) if r % 2 == 0 else (1, 0)):
            setter(args.value if x else args.base)
            for name, fn in (("fwd", fwd), ("bwd", bwd)):
                fn()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
                ev[0].record(st)
                for i in range(args.iters):
                    fn()
                    ev[i + 1].record(st)
                torch.cuda.synchronize()
                res[f"{name}{x}"].append(statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)))
    med = {k: round(statistics.median(v), 4) for k, v in res.items()}
    setter(args.base)
    print(json.dumps({"setter": args.setter, "value": args.value, "base": args.base, "bitwise_equal": equal,
                      "rel_l2_1_vs_0": {k: float(f"{v:.3g}") for k, v in rel.items()}, "median_ms": med,
                      "fwd_1_vs_0": round(med["fwd1"] / med["fwd0"], 4),
                      "bwd_1_vs_0": round(med["bwd1"] / med["bwd0"], 4)}), flush=True)


if __name__ == "__main__":
    main()
