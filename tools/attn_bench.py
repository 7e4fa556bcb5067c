"""Developer A/B of the attention backward at the bench's shapes (JiT-B/16, 1024^2, B=8, 12 heads,
n = 4170 of which 4106 always-valid keys and a masked context tail): the production fused pass
(variant 0) against round 1's split dK/dV + recomputing dQ kernels (variant 9, diagnostic library),
numerics of one against the other and timing (HIP events, interleaved rounds).

  VPT_DIAG=1 python tools/attn_bench.py [--rounds 3]
"""
import os
os.environ.setdefault("VPT_DIAG", "1")  # variant switch lives in libvpt_hip_diag.so only

import argparse
import json
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--n", type=int, default=4170)
    args = ap.parse_args()
    dev = "cuda"
    B, H, n = args.B, 12, args.n
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
    q4, k4, v4 = (ops._t4(qkv, B, rows, H, c) for c in (0, D, 2 * D))
    o4 = ops._t4(o, B, rows, H)
    ws = torch.empty(int(ops.lib.vpt_attn_fused_workspace_bytes(B, H, n)) // 4, device=dev)
    ops.lib.vpt_attn_set_fused_workspace(ws.data_ptr())
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense)
    outs = {}
    for var in (13, 0):
        ops.lib.vpt_attn_set_variant(var)
        gr = [torch.zeros(B * rows, D, dtype=torch.bfloat16, device=dev) for _ in range(3)]
        ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb, *(ops._t4(t, B, rows, H) for t in gr),
                     B, H, rows, n, n_dense)
        outs[var] = gr
    ops.lib.vpt_attn_set_variant(0)
    torch.cuda.synchronize()
    res = {}
    for i, nm in enumerate(("dq", "dk", "dv")):
        a, b = outs[13][i].float(), outs[0][i].float()
        res[f"rel_{nm}_fused_vs_split"] = ((a - b).norm() / b.norm()).item()
        res[f"finite_{nm}"] = bool(torch.isfinite(a).all().item())
    fl = 4.0 * B * H * n * n * 64
    t = {0: [], 13: [], 10: [], 11: [], 12: []}
    for _ in range(args.rounds):
        for var in t:
            ops.lib.vpt_attn_set_variant(var)
            t[var].append(timeit(lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb,
                                                      *(ops._t4(x, B, rows, H) for x in outs[0]), B, H, rows, n,
                                                      n_dense)))
    ops.lib.vpt_attn_set_variant(0)
    tf = timeit(lambda: ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense))
    for var, name in ((13, "fused"), (0, "split_production"), (10, "fused_abl_no_atomics"), (11, "fused_abl_plain_stores"),
                      (12, "fused_abl_no_dq")):
        ms = sorted(t[var])[len(t[var]) // 2]
        res[f"bwd_ms_{name}"] = round(ms, 4)
        res[f"bwd_alg_tflops_{name}"] = round(2 * fl / (ms * 1e-3) / 1e12, 1)
    res["fwd_ms"] = round(tf, 4)
    res["fwd_tflops"] = round(fl / (tf * 1e-3) / 1e12, 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
