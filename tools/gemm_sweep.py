"""Developer sweep: forward GEMM time vs K at fixed tile grids, to split the per-tile cost into a fixed
part (prologue DMA latency + epilogue store) and a per-K part. Prints, per (M, N), the least-squares fit
t_round(K) = a + b*K over 'rounds' of 256 tiles (one 256x256 tile per CU per round).

  python tools/gemm_sweep.py
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def timeit(fn, iters=20):
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
    out = {}
    for (M, N) in ((256 * 64, 1024), (256 * 128, 768), (256 * 128, 2304)):
        tiles = (M // 256) * ((N + 255) // 256)
        rounds = -(-tiles // 256)
        pts = []
        for K in (256, 512, 768, 1536, 2048, 3072):
            x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
            y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ms = timeit(lambda: ops.linear(x, w, out=y))
            us_round = ms * 1e3 / rounds
            pts.append((K, us_round, 2.0 * M * N * K / (ms * 1e-3) / 1e12))
        n = len(pts)
        sx = sum(p[0] for p in pts); sy = sum(p[1] for p in pts)
        sxx = sum(p[0] ** 2 for p in pts); sxy = sum(p[0] * p[1] for p in pts)
        b = (n * sxy - sx * sy) / (n * sxx - sx * sx)
        a = (sy - b * sx) / n
        out[f"{M}x{N}"] = {"tiles": tiles, "rounds": rounds, "fixed_us_per_round": round(a, 2),
                           "us_per_K_per_round": round(b, 5),
                           "steady_TFLOPs": round(256 * 2 * 256 * 256 / (b * 1e-6) / 1e12, 1),
                           "points": [(k, round(u, 2), round(t, 1)) for k, u, t in pts]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
