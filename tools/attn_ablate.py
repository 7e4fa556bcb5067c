"""Developer ablation of the dK/dV backward kernel at the bench shape (diag library): total backward time
per variant (the dQ kernel is unchanged, so differences are the dK/dV kernel's). Variants 4-7 give WRONG
results (timing only): 4 no exp2, 5 4 of the 16 dV/dK MFMAs, 6 no transposed LDS reads, 7 no S/dP LDS reads;
8 = the compiler-scheduled dK/dV body (correct).

  VPT_DIAG=1 python tools/attn_ablate.py
"""
import os
os.environ.setdefault("VPT_DIAG", "1")
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--vars", default="0,4,5,6,7,8", help="vpt_attn_set_variant values (diag dispatcher)")
    args = ap.parse_args()
    dev = "cuda"
    B, H, n = 8, 12, 4170
    rows, D = n, 768
    n_dense = n - 64
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * rows, 3 * D, device=dev, generator=g).bfloat16()
    qkv[:, :D] = (qkv[:, :D].float() * ops.attn_q_scale(0.125)).bfloat16()
    kb = torch.zeros(B, rows, device=dev)
    o = torch.empty(B * rows, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, rows, device=dev)
    delta = torch.empty_like(lse)
    do = torch.randn(B * rows, D, device=dev, generator=g).bfloat16()
    gr = [torch.zeros(B * rows, D, dtype=torch.bfloat16, device=dev) for _ in range(3)]
    q4, k4, v4 = (ops._t4(qkv, B, rows, H, c) for c in (0, D, 2 * D))
    o4 = ops._t4(o, B, rows, H)
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense)
    res = {}
    for r in range(3):
        for var in [int(v) for v in args.vars.split(",")]:
            ops.lib.vpt_attn_set_variant(var)
            ms = timeit(lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb,
                                             *(ops._t4(t, B, rows, H) for t in gr), B, H, rows, n, n_dense))
            res.setdefault(var, []).append(ms)
    ops.lib.vpt_attn_set_variant(0)
    # current diag dispatcher (diag_attn_bwd_variants): 0 production one-launch; split pair: 7 compiler-scheduled
    # dK/dV (correct), 1 no next-tile staging in either loop (wrong), 2 row reads for the transposes (wrong),
    # 3-6 dK/dV ablations (wrong)
    print(json.dumps({f"variant{k}": round(sorted(v)[1], 4) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
