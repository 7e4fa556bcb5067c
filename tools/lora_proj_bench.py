"""Standalone timing of the rank-16 LoRA projection kernel (vpt_lora_proj) at the config-5 shapes, both W
layouts (down [16][K] k-major; up [K][16]), against the bytes it must read (X once): us per call and GB/s.

  python tools/lora_proj_bench.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def timeit(fn, iters=50):
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
    out = {}
    flush = torch.empty(512 * 1024 * 1024 // 4, dtype=torch.float32, device=dev)  # > Infinity Cache
    for M, K in [(4096, 1280), (4096, 5120), (4096, 10240), (16384, 640), (16384, 2560), (924, 1280)]:
        x = torch.randn(M, K, device=dev).bfloat16()
        down = (torch.randn(16, K, device=dev) * 0.05).bfloat16()
        up = (torch.randn(K, 16, device=dev) * 0.05).bfloat16()
        y = torch.empty(M, 16, dtype=torch.bfloat16, device=dev)
        for name, w, km in (("down", down, True), ("up", up, False)):
            warm = sorted(timeit(lambda: ops.lora_proj(x, w, km, y)) for _ in range(5))[2]

            def cold():
                flush.zero_()
                ops.lora_proj(x, w, km, y)
            t_cold = timeit(cold, 20) - timeit(lambda: flush.zero_(), 20)
            out[f"M{M}_K{K}_{name}"] = {"warm_us": round(warm, 2), "cold_us": round(t_cold, 2),
                                        "warm_GBps": round(M * K * 2 / warm / 1e3, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
