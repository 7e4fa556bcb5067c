"""Split-K sweep of the JiT-B/16 weight gradients (vpt_linear_wgrad with the fused bias gradient, as the engine calls
it) at the token counts of the C3 (B=8 1024^2) and C2 (B=16 512^2) steps: time per split count against the one
ops.wgrad_splits picks. Interleaved rounds, medians, HIP events on the launching stream.

  python tools/wgrad_split_sweep.py [--rounds 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = "cuda"
    D, F = 768, 2048
    shapes = [(2 * F, D), (3 * D, D), (D, F), (D, D), (768, D)]  # (N out, K in): W12, Wqkv, W3, Wo, final
    out = {}
    for M in (16 * 1104, 8 * 4170):
        for N, K in shapes:
            dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            dw = torch.empty(N, K, device=dev)
            db = torch.empty(N, device=dev)
            cands = sorted({s for s in (1, 2, 3, 4, 5, 6, 8, 10, 12, 14, 16, 20, 24, 28, 32, 40) if M // s >= 256})
            ws = torch.empty(max(ops.linear_wgrad_workspace_bytes(M, N, K, s) for s in cands) // 4 + 1, device=dev)
            t = {s: [] for s in cands}
            for _ in range(args.rounds):
                for s in cands:
                    t[s].append(timeit(lambda: ops.linear_wgrad(dy, x, dw, splits=s, workspace=ws, bias_out=db)))
            med = {s: sorted(v)[len(v) // 2] for s, v in t.items()}
            pick = ops.wgrad_splits(N, K, M)
            best = min(med, key=med.get)
            out[f"M{M} N{N} K{K}"] = {"model_splits": pick, "model_us": round(med.get(pick, float("nan")), 1),
                                      "best_splits": best, "best_us": round(med[best], 1),
                                      "us": {s: round(v, 1) for s, v in med.items()}}
            print(json.dumps({f"M{M} N{N} K{K}": out[f"M{M} N{N} K{K}"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
