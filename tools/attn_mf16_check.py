"""Numerics of the attention backward's 16x16x32 bodies (diagnostic library, vpt_attn_set_bwd_mfma16: bit 1 dK/dV,
bit 2 dQ) against the fp32 torch reference, at the shapes of tests/test_kernels_gpu.py::test_attention_fwd_bwd (ragged
lengths, context / padding key bias, partial query and key tiles) and a cross-attention shape (nk != n); every mask
0..3 reports the relative L2 error of dq, dk, dv (the tests' bar: 2e-2).

  python tools/attn_mf16_check.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402

DEV = torch.device("cuda", 0)


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * scale).bfloat16()


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def case(n, nk, n_dense, masked, B=2, H=3):
    rq, rk = (n + 127) // 128 * 128, (nk + 127) // 128 * 128
    D = 64 * H
    q = rnd(B * rq, D, seed=40).float() * ops.attn_q_scale(0.125)
    q = q.bfloat16()
    kv = rnd(B * rk, 2 * D, seed=41)
    kb = torch.zeros(B, rk, device=DEV)
    if masked:
        kb[:, n_dense + (nk - n_dense) // 2:] = float("-inf")
        kb[1, n_dense:] = 0.0
    o = torch.zeros(B * rq, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B, H, rq, device=DEV)
    q4, k4, v4 = ops._t4(q, B, rq, H, 0), ops._t4(kv, B, rk, H, 0), ops._t4(kv, B, rk, H, D)
    ops.attn_fwd(q4, k4, v4, ops._t4(o, B, rq, H, 0), lse, kb, B, H, rq, n, n_dense, nk=nk)
    do = rnd(B * rq, D, seed=42)

    def heads(t, r, c0, nn):
        return t[:, c0:c0 + D].float().view(B, r, H, 64)[:, :nn].permute(0, 2, 1, 3).contiguous()

    qf = (heads(q, rq, 0, n) / ops.attn_q_scale(0.125)).requires_grad_(True)
    kf = heads(kv, rk, 0, nk).requires_grad_(True)
    vf = heads(kv, rk, D, nk).requires_grad_(True)
    s = torch.einsum("bhqd,bhkd->bhqk", qf, kf) * 0.125 + kb[:, None, None, :nk]
    ref = torch.einsum("bhqk,bhkd->bhqd", torch.softmax(s, -1), vf)
    ref.backward(heads(do, rq, 0, n))
    out = {}
    for mask in (0, 1, 2, 3, 7, 15):
        _lib.lib.vpt_attn_set_bwd_mfma16(mask)
        dq = torch.zeros(B * rq, D, dtype=torch.bfloat16, device=DEV)
        dkv = torch.zeros(B * rk, 2 * D, dtype=torch.bfloat16, device=DEV)
        delta = torch.zeros(B, H, rq, device=DEV)
        ops.attn_bwd(q4, k4, v4, ops._t4(o, B, rq, H, 0), ops._t4(do, B, rq, H, 0), lse, delta, kb,
                     ops._t4(dq, B, rq, H, 0), ops._t4(dkv, B, rk, H, 0), ops._t4(dkv, B, rk, H, D), B, H, rq, n,
                     n_dense, nk=nk)
        torch.cuda.synchronize()
        out[mask] = {"dq": rel(heads(dq, rq, 0, n), qf.grad),
                     "dk": rel(heads(dkv, rk, 0, nk), kf.grad), "dv": rel(heads(dkv, rk, D, nk), vf.grad),
                     "finite": bool(torch.isfinite(dq).all() and torch.isfinite(dkv).all())}
    _lib.lib.vpt_attn_set_bwd_mfma16(0)
    return out


def main():
    _lib.use_diag()
    worst = 0.0
    for n, nk, nd, masked in ((200, 200, 150, True), (330, 330, 330, False), (64, 64, 40, True),
                              (1034, 1034, 1024, True), (700, 700, 520, True), (300, 77, 77, False),
                              (257, 520, 400, True)):
        r = case(n, nk, nd, masked)
        for m, v in r.items():
            if m:
                worst = max(worst, v["dq"], v["dk"], v["dv"], 0.0 if v["finite"] else 1.0)
        print(json.dumps({"n": n, "nk": nk, "n_dense": nd, "masked": masked,
                          "rel": {m: {k: (round(x, 5) if isinstance(x, float) else x) for k, x in v.items()}
                                  for m, v in r.items()}}), flush=True)
    print(json.dumps({"worst_rel_16x16": worst, "ok": worst < 2e-2}))


if __name__ == "__main__":
    main()
