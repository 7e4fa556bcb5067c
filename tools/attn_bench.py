"""Developer A/B of the attention backward at the bench's shapes (JiT-B/16, 1024^2, B=8, 12 heads,
n = 4170 of which 4106 always-valid keys and a masked context tail): the 64-rows-per-wave dK/dV + dQ
pair (production) against the 32-row pair (diagnostic library switch vpt_attn_set_rows64), numerics of
one against the other and timing (HIP events, interleaved rounds).

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
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense)
    outs = {}
    for r64 in (0, 1, 2, 4, 3):  # 32-row pair vs 64-row variants (bit mask), same inputs
        ops.lib.vpt_attn_set_rows64(r64)
        gr = [torch.zeros(B * rows, D, dtype=torch.bfloat16, device=dev) for _ in range(3)]
        ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb, *(ops._t4(t, B, rows, H) for t in gr),
                     B, H, rows, n, n_dense)
        outs[r64] = gr
    torch.cuda.synchronize()
    res = {}
    for i, nm in enumerate(("dq", "dk", "dv")):
        for r64 in (1, 2, 4, 3):
            a, b = outs[r64][i].float(), outs[0][i].float()
            res[f"rel_{nm}_v{r64}_vs_rows32"] = ((a - b).norm() / b.norm()).item()
    fl = 4.0 * B * H * n * n * 64
    t = {0: [], 1: [], 2: [], 4: [], 3: []}
    for _ in range(args.rounds):
        for r64 in t:
            ops.lib.vpt_attn_set_rows64(r64)
            t[r64].append(timeit(lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb,
                                                      *(ops._t4(x, B, rows, H) for x in outs[0]), B, H, rows, n,
                                                      n_dense)))
    ops.lib.vpt_attn_set_rows64(0)
    tf = timeit(lambda: ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense))
    for r64, name in ((0, "rows32"), (1, "dkdv64"), (2, "dq64_occ2"), (4, "dq64_occ1"), (3, "dkdv64_dq64occ2")):
        ms = sorted(t[r64])[len(t[r64]) // 2]
        res[f"bwd_ms_{name}"] = round(ms, 4)
        res[f"bwd_alg_tflops_{name}"] = round(2 * fl / (ms * 1e-3) / 1e12, 1)
    res["fwd_ms"] = round(tf, 4)
    res["fwd_tflops"] = round(fl / (tf * 1e-3) / 1e12, 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
