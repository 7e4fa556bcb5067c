"""Config 5's rank-16 row-block kernels (16 rows per workgroup) at M = 4096 (256 row blocks: one per CU) and at the
bucketed M = 4224 (264 row blocks: 8 CUs take a second one) -- is the launch time a second round of blocks?
HIP-event medians per launch, GB/s of the algorithmic bytes.

  python tools/c5_lora_tail_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def timeit(fn, iters=20, rounds=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(rounds):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(out)[len(out) // 2]


def main():
    dev = "cuda"
    res = {}
    for M, F in ((4096, 5120), (4224, 5120), (6144, 5120), (8192, 5120), (16384, 2560), (16896, 2560)):
        dy = torch.randn(M, F, device=dev).bfloat16()
        x12 = torch.randn(M, 2 * F, device=dev).bfloat16()
        up = (torch.randn(2 * F, 16, device=dev) * 0.05).bfloat16()
        vs = torch.empty(M, 16, dtype=torch.bfloat16, device=dev)
        gg = torch.randn(M, F, device=dev).bfloat16()
        down = (torch.randn(16, F, device=dev) * 0.05).bfloat16()
        x = torch.randn(M, 1280, device=dev).bfloat16()
        down1 = (torch.randn(16, 1280, device=dev) * 0.05).bfloat16()
        ds = torch.empty(M, 16, dtype=torch.bfloat16, device=dev)
        r = {
            "geglu_bwd_lora": (timeit(lambda: ops.geglu_bwd_lora(dy, x12, up, 0.0625, vs)), M * F * 2 * 5),
            "geglu_bwd": (timeit(lambda: ops.geglu_bwd(dy, x12)), M * F * 2 * 5),
            "geglu_fwd": (timeit(lambda: ops.geglu_fwd(x12)), M * F * 2 * 3),
            "lora_proj_K5120": (timeit(lambda: ops.lora_proj(gg, down, True, ds)), M * F * 2),
            "lora_proj_K1280": (timeit(lambda: ops.lora_proj(x, down1, True, ds)), M * 1280 * 2),
            "lora_proj_up_K2F": (timeit(lambda: ops.lora_proj(x12, up, False, ds)), M * 2 * F * 2),
        }
        r["lora_proj_up_K2F+geglu_bwd"] = (r["lora_proj_up_K2F"][0] + r["geglu_bwd"][0], M * F * 2 * 7)
        res[f"{M}x{F}"] = {k: {"us": round(t, 1), "GB/s": round(b / t / 1e3, 0)} for k, (t, b) in r.items()}
        print(json.dumps({f"{M}x{F}": res[f"{M}x{F}"]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
