"""Attention kernels alone at the C3 shape (JiT-B/16, B=8, 1024^2: n = 4170 rows, 4106 always-valid keys, 12 heads,
QK-normed inputs) -- forward (online maximum and fixed reference), backward (plain and with the fused QK-norm
backward) -- `--iters` launches each, for rocprofv3 counter passes over exactly these kernels.

  python tools/attn_shape_run.py [--iters 5]
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
    ap.add_argument("--xcd", type=int, default=None, help="block order (diagnostic library): 1 XCD-contiguous, 0 linear")
    ap.add_argument("--only", default=None, help="run only the fwd_qknorm and plain bwd launches")
    args = ap.parse_args()
    if args.xcd is not None:
        from vpt import _lib
        _lib.use_diag()
        _lib.lib.vpt_attn_set_xcd_order(args.xcd)
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
    dqkv = torch.zeros(M, 3 * D, dtype=torch.bfloat16, device=dev)
    dqk = torch.zeros(M, 2 * D, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B, H, n, device=dev)
    part = torch.empty(ops.attn_bwd_dw_rows(B, H, n), 128, device=dev)
    q4, k4, v4 = ops._t4(qk, B, n, H, 0), ops._t4(qk, B, n, H, D), ops._t4(qkv, B, n, H, 2 * D)
    o4, do4 = ops._t4(o, B, n, H, 0), ops._t4(do, B, n, H, 0)
    for _ in range(0 if args.only else args.iters):
        ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, n, n, nd)
    for _ in range(args.iters):
        ops.attn_fwd_qknorm(q4, k4, v4, o4, lse, kb, wq, wk, B, H, n, n, nd)
    for _ in range(args.iters):
        ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                     ops._t4(dqkv, B, n, H, 2 * D), B, H, n, n, nd)
    for _ in range(0 if args.only else args.iters):
        ops.attn_bwd_qknorm(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(qkv, B, n, H, 0), ops._t4(qkv, B, n, H, D),
                            wq, wk, cos, sin, ops._t4(dqkv, B, n, H, 0), ops._t4(dqkv, B, n, H, D), part,
                            ops._t4(dqkv, B, n, H, 2 * D), B, H, n, n, nd)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
