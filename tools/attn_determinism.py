"""Run-to-run determinism of the attention backward at the C3 shape (JiT-B/16, B=8, 1024^2: n = 4170 rows, 4106
always-valid keys, 12 heads, QK-normed inputs): one forward, then the backward `--runs` times on identical inputs; every
run's dq / dk / dv is compared bitwise with the first, and differing elements are located (batch, head, row range,
magnitude). `--lib NAME` uses lib/var/libvpt_hip_NAME.so, `--diag-setter S --diag-value V` a diagnostic switch.

  python tools/attn_determinism.py [--runs 6] [--fresh]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--fresh", action="store_true", help="zero the outputs before every run")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--diag-setter", default=None)
    ap.add_argument("--diag-value", type=int, default=0)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--fwd-each", action="store_true", help="re-run the forward before every backward")
    ap.add_argument("--torch-between", action="store_true",
                    help="fp32 torch attention of two heads between forward and backward (tools/lib_ab.py's check)")
    args = ap.parse_args()
    if args.lib:
        from tools.lib_ab import lib_path
        _lib.use_library(lib_path(args.lib))
    if args.diag_setter:
        _lib.use_diag()
        getattr(_lib.lib, args.diag_setter)(args.diag_value)
    dev = torch.device("cuda", 0)
    B, H, n, nd = args.B, 12, 4170, 4106
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
    def torch_work():
        for h in range(2):
            q = qk[:n, h * 64:(h + 1) * 64].float()
            k = qk[:n, D + h * 64:D + (h + 1) * 64].float()
            v = qkv[:n, 2 * D + h * 64:2 * D + (h + 1) * 64].float()
            s = q @ k.T + kb[0][None, :]
            torch.softmax(s * 0.6931471805599453, 1) @ v

    ops.attn_fwd_qknorm(q4, k4, v4, o4, lse, kb, wq, wk, B, H, n, n, nd)
    torch.cuda.synchronize()
    outs = []
    for r in range(args.runs):
        if args.fresh:
            dqk.zero_()
            dqkv.zero_()
        if args.fwd_each and r > 0:
            ops.attn_fwd_qknorm(q4, k4, v4, o4, lse, kb, wq, wk, B, H, n, n, nd)
            torch.cuda.synchronize()
        if args.torch_between:
            torch_work()
        ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                     ops._t4(dqkv, B, n, H, 2 * D), B, H, n, n, nd)
        torch.cuda.synchronize()
        outs.append({"dq": dqk[:, :D].clone(), "dk": dqk[:, D:].clone(), "dv": dqkv[:, 2 * D:].clone(),
                     "delta": delta.clone(), "o": o.clone(), "lse": lse.clone()})
    rep = []
    for r in range(1, args.runs):
        row = {}
        for k in ("dq", "dk", "dv", "delta", "o", "lse"):
            a, b = outs[0][k].float(), outs[r][k].float()
            ne = a != b
            cnt = int(ne.sum())
            ent = {"differ": cnt}
            if cnt and k not in ("delta", "lse"):
                idx = ne.nonzero()
                rows, cols = idx[:, 0], idx[:, 1]
                bb, rr, hh = rows // n, rows % n, cols // 64
                ent.update(batches=sorted(set(bb.tolist()))[:8], heads=sorted(set(hh.tolist()))[:12],
                           row_min=int(rr.min()), row_max=int(rr.max()), n_rows=int(torch.unique(rows).numel()),
                           max_abs=float((a - b).abs().max()), ref_abs_max=float(a.abs().max()),
                           rel_l2=float((a - b).norm() / a.norm()))
            row[k] = ent
        rep.append(row)
        print(f"run {r}: " + json.dumps(row), flush=True)
    print(json.dumps({"runs": args.runs, "fresh": args.fresh, "B": B, "report": rep}))


if __name__ == "__main__":
    main()
