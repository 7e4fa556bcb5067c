"""The JiT-B/16 Linear shapes that do not carry a fused SwiGLU / QK-norm epilogue, at the C3 (B=8 1024^2) and C2
(B=16 512^2) token counts: the 256x256 ring (geometry 256) against 128x128 tiles on the R2 pipeline (geometry 1281),
bf16 output with the residual where the step has one. Interleaved rounds, medians of HIP-event times; outputs compared.

  python tools/r2_128_c3_probe.py [--rounds 5]
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
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = "cuda"
    res = {}
    # (N, K, direction, residual): o-proj fwd, W3 fwd, qkv dgrad, o-proj dgrad, W3 dgrad... (dgrad = dY . W)
    shapes = [(768, 768, "fwd", True), (768, 2048, "fwd", True), (768, 2304, "dgrad", False),
              (768, 768, "dgrad", False), (768, 4096, "dgrad", False)]
    for M in (8 * 4154, 16 * 1104):
        for N, K, kind, res_on in shapes:
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.03).to(torch.bfloat16) if kind == "fwd" else \
                (torch.randn(K, N, device=dev) * 0.03).to(torch.bfloat16)
            resid = torch.randn(M, N, device=dev).to(torch.bfloat16) if res_on else None
            outs = {g: torch.empty(M, N, dtype=torch.bfloat16, device=dev) for g in (256, 1281)}
            t = {g: [] for g in outs}
            for _ in range(args.rounds):
                for g in outs:
                    t[g].append(timeit(lambda: ops.gemm(a, True, w, kind == "fwd", M, N, K, outs[g], resid=resid,
                                                        geometry=g)))
            key = f"{kind} M{M} N{N} K{K}"
            res[key] = {"us": {str(g): round(sorted(v)[len(v) // 2], 1) for g, v in t.items()},
                        "maxdiff": (outs[256].float() - outs[1281].float()).abs().max().item()}
            print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
