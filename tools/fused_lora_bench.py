"""Standalone per-call time of the fused LayerNorm + LoRA-down kernel against the pair it replaces
(layernorm_fwd + lora_proj(_grouped)) at the config-5 shapes, launch overhead included. Prints JSON (us per call).

  python tools/fused_lora_bench.py
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
    return round(s.elapsed_time(e) / iters * 1e3, 2)


def main():
    dev = "cuda"
    res = {}
    for M, D, G in [(4096, 1280, 3), (4096, 1280, 1), (16384, 640, 3)]:
        x = torch.randn(M, D, device=dev).bfloat16()
        w = torch.ones(D, device=dev).bfloat16()
        b = torch.zeros(D, device=dev).bfloat16()
        down = (torch.randn(16 * G, D, device=dev) * 0.05).bfloat16()
        ds = torch.empty(M, 16 * G, dtype=torch.bfloat16, device=dev)
        res[f"ln_M{M}_D{D}_G{G}"] = {
            "fused": timeit(lambda: ops.layernorm_lora_fwd(x, w, b, down, G, 0.0625, ds)),
            "pair": timeit(lambda: ops.lora_proj_grouped(ops.layernorm_fwd(x, w, b)[0], 0, down, 16 * D, G, True, ds)),
            "ln_only": timeit(lambda: ops.layernorm_fwd(x, w, b))}
    for M, F in [(4096, 5120), (16384, 2560)]:
        dy = torch.randn(M, F, device=dev).bfloat16()
        x12 = torch.randn(M, 2 * F, device=dev).bfloat16()
        up = (torch.randn(2 * F, 16, device=dev) * 0.05).bfloat16()
        vs = torch.empty(M, 16, dtype=torch.bfloat16, device=dev)
        dx12 = torch.empty_like(x12)
        res[f"geglu_bwd_M{M}_F{F}"] = {
            "fused": timeit(lambda: ops.geglu_bwd_lora(dy, x12, up, 0.0625, vs, dx12=dx12)),
            "pair": timeit(lambda: ops.lora_proj(ops.geglu_bwd(dy, x12, dx12), up, False, vs, alpha=0.0625)),
            "geglu_bwd_only": timeit(lambda: ops.geglu_bwd(dy, x12, dx12))}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
