"""Wave quantisation of the N = 768 ring GEMMs: time per call against M (row tiles of 256; items = row tiles x 3 on
256 persistent blocks), for the W1|W2 input gradient (K = 4096), the W3 forward (K = 2048, residual epilogue) and the
q|k|v input gradient (K = 2304). A staircase at multiples of 85.3 row tiles means the partial last round costs a full
round; a straight line means it runs proportionally faster.

  python tools/gemm_rounds_probe.py
"""
import json
import os
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
    dev = "cuda"
    N = 768
    Mmax = 176 * 256
    res = {}
    for name, K in (("w12_dgrad_K4096", 4096), ("w3_fwd_K2048", 2048), ("qkv_dgrad_K2304", 2304)):
        w = (torch.randn(K, N, device=dev) * 0.05).bfloat16() if "dgrad" in name else \
            (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        a = torch.randn(Mmax, K, device=dev).bfloat16()
        r = torch.randn(Mmax, N, device=dev).bfloat16()
        b = (torch.randn(N, device=dev) * 0.05).bfloat16()
        y = torch.empty(Mmax, N, dtype=torch.bfloat16, device=dev)
        row = {}
        for tiles in range(64, 177, 4):
            M = tiles * 256
            if "dgrad" in name:
                fn = lambda: ops.linear_dgrad(a[:M], w, out=y[:M])  # noqa: E731
            else:
                fn = lambda: ops.linear(a[:M], w, b, resid=r[:M], out=y[:M])  # noqa: E731
            row[tiles] = round(timeit(fn), 2)
        res[name] = row
        print(name, json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
