"""NF4 GEMM at the C5 shapes: TFLOP/s of vpt_gemm_nf4 (forward / input-gradient, with the LoRA tile), its
timing ablations (diag library: no dequant, no code loads), and the bf16 T128 / ring GEMM on the dequantised
weight beside it. VPT_DIAG=1 python tools/nf4_bench.py"""
import os
os.environ.setdefault("VPT_DIAG", "1")
import json
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
import torch  # noqa: E402

from vpt import ops  # noqa: E402
from vpt.sdxl import NF4Weight, dynamic_map  # noqa: E402


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
    dev = "cuda"
    code2 = dynamic_map().to(dev)
    shapes = {"640_qkvo": (16384, 640, 640), "640_ffproj": (16384, 5120, 640), "640_ffout": (16384, 640, 2560),
              "1280_qkvo": (4096, 1280, 1280), "1280_ffproj": (4096, 10240, 1280), "1280_ffout": (4096, 1280, 5120)}
    res = {}
    for name, (M, N, K) in shapes.items():
        w = NF4Weight.quantize((torch.randn(N, K, device=dev) / K ** 0.5).bfloat16(), code2)
        wd = w.dequantize()
        x = torch.randn(M, K, device=dev).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        la, lb_f, lb_d = (torch.randn(M, 16, device=dev).bfloat16(), torch.randn(N, 16, device=dev).bfloat16(),
                          torch.randn(16, K, device=dev).bfloat16())
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        fl = 2.0 * M * N * K
        r = {}
        for abl in (0, 1, 2):
            ops.lib.vpt_gemm_set_nf4_ablation(abl)
            r[f"fwd_abl{abl}"] = fl / (timeit(lambda: ops.gemm_nf4(x, w, True, y, lora_a=la, lora_b=lb_f)) * 1e-3) / 1e12
            r[f"dgrad_abl{abl}"] = fl / (timeit(lambda: ops.gemm_nf4(dy, w, False, dx, lora_a=la, lora_b=lb_d)) * 1e-3) / 1e12
        ops.lib.vpt_gemm_set_nf4_ablation(0)
        r["bf16_t128_fwd"] = fl / (timeit(lambda: ops.gemm(x, True, wd, True, M, N, K, y, geometry=128)) * 1e-3) / 1e12
        r["bf16_auto_fwd"] = fl / (timeit(lambda: ops.linear(x, wd, out=y)) * 1e-3) / 1e12
        res[name] = {k: round(v, 1) for k, v in r.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
