"""A diagnostic variant of the attention backward against the production kernel at the C3 shape: bitwise equality of
dq / dk / dv, then interleaved HIP-event timing (medians).
  --knob stages --value 3: 3-stage LDS rings (vpt_attn_set_bwd_stages)

  python tools/attn_bwd_variant_check.py --knob stages --value 3 [--rounds 6]
"""
import os
import argparse  # noqa: E402
import json  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402

_lib.use_diag()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--knob", choices=("stages",), default="stages")
    ap.add_argument("--value", type=int, default=3)
    args = ap.parse_args()
    setter = _lib.lib.vpt_attn_set_bwd_stages
    base = 2
    A, Bv = base, args.value
    dev = torch.device("cuda", 0)
    B, H, n, nd = 8, 12, 4170, 4106
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
    q4, k4, v4 = ops._t4(qk, B, n, H, 0), ops._t4(qk, B, n, H, D), ops._t4(qkv, B, n, H, 2 * D)
    o4, do4 = ops._t4(o, B, n, H, 0), ops._t4(do, B, n, H, 0)
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, n, n, nd)
    outs = {}

    def bwd(val):
        setter(val)
        dqk = torch.zeros(M, 2 * D, dtype=torch.bfloat16, device=dev)
        dv = torch.zeros(M, D, dtype=torch.bfloat16, device=dev)
        delta = torch.empty(B, H, n, device=dev)
        ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                     ops._t4(dv, B, n, H, 0), B, H, n, n, nd)
        return dqk, dv
    for st in (A, Bv):
        outs[st] = bwd(st)
    torch.cuda.synchronize()
    eq = all(torch.equal(a, b) for a, b in zip(outs[A], outs[Bv]))
    times = {A: [], Bv: []}
    for r in range(args.rounds):
        for st in ((A, Bv) if r % 2 == 0 else (Bv, A)):
            setter(st)
            dqk = torch.zeros(M, 2 * D, dtype=torch.bfloat16, device=dev)
            dv = torch.zeros(M, D, dtype=torch.bfloat16, device=dev)
            delta = torch.empty(B, H, n, device=dev)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(3):
                ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                             ops._t4(dv, B, n, H, 0), B, H, n, n, nd)
            e.record()
            torch.cuda.synchronize()
            times[st].append(s.elapsed_time(e) / 3)
    med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
    setter(base)
    print(json.dumps({"knob": args.knob, "bitwise_equal": eq, "ms": {k: [round(x, 4) for x in v] for k, v in times.items()},
                      "median_ms": med}))


if __name__ == "__main__":
    main()
