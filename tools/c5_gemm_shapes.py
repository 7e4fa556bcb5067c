"""Developer microbenchmark: the config-5 (SDXL QLoRA) base+LoRA GEMM shapes (forward and input gradient of
every LoRA target at the 1280-channel / 32x32 and 640-channel / 64x64 stages, B = 4), vpt_gemm_bf16_lora in
both geometries, the plain GEMM with split-K (no LoRA) and torch.matmul (hipBLASLt) beside them. Median of
interleaved rounds, TFLOP/s and us per call, one JSON object.   python tools/c5_gemm_shapes.py"""
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
    dev = "cuda"
    # (name, M, N_out, K_in, per-step count): forward computes [M, N_out] over K_in; dgrad [M, K_in] over N_out
    shapes = [("1280.qkvo", 4096, 1280, 1280, 360), ("1280.ff0", 4096, 10240, 1280, 60), ("1280.ff2", 4096, 1280, 5120, 60),
              ("1280.kv", 924, 1280, 2048, 120), ("640.qkvo", 16384, 640, 640, 60), ("640.ff0", 16384, 5120, 640, 10),
              ("640.ff2", 16384, 640, 2560, 10), ("640.kv", 924, 640, 2048, 20)]
    res = {}
    for name, M, No, Ki, cnt in shapes:
        W = (torch.randn(No, Ki, device=dev) * 0.03).bfloat16()
        for fwd in (True, False):
            if name.endswith(".kv") and not fwd:
                continue  # the context needs no gradient
            N, K = (No, Ki) if fwd else (Ki, No)
            a = torch.randn(M, K, device=dev).bfloat16()
            a2 = torch.randn(M, 16, device=dev).bfloat16()
            b2 = (torch.randn(N, 16, device=dev) if fwd else torch.randn(16, N, device=dev)).bfloat16()
            out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            fl = 2.0 * M * N * K
            r = {"count_per_step": cnt}
            for geo in (128, 256):
                ms = timeit(lambda: ops.gemm_lora(a, W, fwd, a2, b2, M, N, K, out, geometry=geo))
                r[f"lora_g{geo}"] = [round(fl / ms / 1e9, 1), round(ms * 1e3, 1)]
            for sp in (2, 3, 4):
                ws = torch.empty(sp * M * N, dtype=torch.float32, device=dev)
                ms = timeit(lambda: ops.gemm(a, True, W, fwd, M, N, K, out, splits=sp, workspace=ws, geometry=256))
                r[f"splitk{sp}_g256"] = [round(fl / ms / 1e9, 1), round(ms * 1e3, 1)]
                ms = timeit(lambda: ops.gemm_lora(a, W, fwd, a2, b2, M, N, K, out, geometry=128, splits=sp))
                r[f"lora_splitk{sp}_g128"] = [round(fl / ms / 1e9, 1), round(ms * 1e3, 1)]
            Wt = W.t() if fwd else W
            ms = timeit(lambda: torch.matmul(a, Wt))
            r["torch"] = [round(fl / ms / 1e9, 1), round(ms * 1e3, 1)]
            res[f"{name}.{'fwd' if fwd else 'dgrad'} M{M} N{N} K{K}"] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
