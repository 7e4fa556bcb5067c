"""Split-K sweep of the weight-gradient ring GEMM (vpt_linear_wgrad, fused bias) at the JiT-B/16 B=8 1024^2
shapes: median us per call for each split count against ops.wgrad_splits' choice. One JSON object.

  python tools/wgrad_sweep.py [--rounds 3]
"""
import argparse
import json
import os
import statistics
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
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    M = 8 * 4170
    shapes = {"qkv": (2304, 768), "o": (768, 768), "w12": (4096, 768), "w3": (768, 2048)}
    g = torch.Generator(device="cuda").manual_seed(0)
    out = {}
    for name, (N, K) in shapes.items():
        dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        dw = torch.empty(N, K, device="cuda")
        db = torch.empty(N, device="cuda")
        pick = ops.wgrad_splits(N, K, M)
        cands = sorted({1, 2, 3, 4, 6, 8, 10, 12, 16, pick} | {max(1, pick - 1), pick + 1})
        ws = torch.empty(max(ops.linear_wgrad_workspace_bytes(M, N, K, s) for s in cands) // 4 + 1, device="cuda")
        res = {}
        for _ in range(args.rounds):
            for s in cands:
                res.setdefault(s, []).append(
                    timeit(lambda: ops.linear_wgrad(dy, x, dw, splits=s, workspace=ws, bias_out=db)))
        out[name] = {"pick": pick, "us": {str(s): round(statistics.median(v), 1) for s, v in res.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
