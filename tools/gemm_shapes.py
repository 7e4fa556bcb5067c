"""Developer microbenchmark at HEAD: the production GEMM entry points at the JiT-B/16 1024^2 B=8 shapes
(fwd / dgrad / wgrad of every block Linear, the fused SwiGLU forward and backward vs their unfused
pairs), torch.matmul (hipBLASLt) beside them as a reference bar. Random (gaussian) data, interleaved
rounds in one process, median per entry. Prints one JSON object (TFLOP/s and us per call).

  python tools/gemm_shapes.py [--rounds 3] [--M 33360]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--M", type=int, default=8 * 4170)
    args = ap.parse_args()
    dev = "cuda"
    M, D, F = args.M, 768, 2048
    res: dict = {}

    def put(name, fl, ms):
        res.setdefault(name, []).append((fl / (ms * 1e-3) / 1e12, ms * 1e3))

    ws = torch.empty(64 * 4096 * 2048, dtype=torch.float32, device=dev)
    shapes = {"qkv": (3 * D, D), "o": (D, D), "w12": (2 * F, D), "w3": (D, F)}
    for _ in range(args.rounds):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
            b = (torch.randn(N, device=dev) * 0.05).bfloat16()
            dy = torch.randn(M, N, device=dev).bfloat16()
            y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
            dw = torch.empty(N, K, dtype=torch.float32, device=dev)
            fl = 2.0 * M * N * K
            sp = ops.wgrad_splits(N, K, M)
            put(f"{name}.fwd", fl, timeit(lambda: ops.linear(x, w, b, out=y)))
            if K == N or name == "w3":  # residual epilogue (O / W3 projections)
                r = torch.randn(M, N, device=dev).bfloat16()
                put(f"{name}.fwd_resid", fl, timeit(lambda: ops.linear(x, w, b, resid=r, out=y)))
            put(f"{name}.dgrad", fl, timeit(lambda: ops.linear_dgrad(dy, w, out=dx)))
            put(f"{name}.wgrad_s{sp}", fl, timeit(lambda: ops.linear_wgrad(dy, x, dw, splits=sp, workspace=ws)))
            put(f"{name}.bias_grad", fl, timeit(lambda: ops.bias_grad(dy, b.float())))
            put(f"{name}.torch_fwd", fl, timeit(lambda: torch.matmul(x, w.t())))
            put(f"{name}.torch_dgrad", fl, timeit(lambda: torch.matmul(dy, w)))
        # fused SwiGLU forward vs GEMM + elementwise
        x = torch.randn(M, D, device=dev).bfloat16()
        w12 = (torch.randn(2 * F, D, device=dev) * 0.05).bfloat16()
        b12 = (torch.randn(2 * F, device=dev) * 0.05).bfloat16()
        x12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=dev)
        h = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
        fl = 2.0 * M * 2 * F * D
        put("swiglu_fwd.fused", fl, timeit(lambda: ops.linear_swiglu(x, w12, b12, x12, h)))
        put("swiglu_fwd.unfused", fl, timeit(lambda: (ops.linear(x, w12, b12, out=x12), ops.swiglu_fwd(x12, h))))
        put("swiglu_fwd.elementwise_only", fl, timeit(lambda: ops.swiglu_fwd(x12, h)))
        # fused SwiGLU backward (W3 dgrad + derivative) vs dgrad + elementwise
        dy = torch.randn(M, D, device=dev).bfloat16()
        w3 = (torch.randn(D, F, device=dev) * 0.05).bfloat16()
        dx12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=dev)
        dh = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
        fl = 2.0 * M * F * D
        put("swiglu_bwd.fused", fl, timeit(lambda: ops.linear_dgrad_swiglu(dy, w3, x12, dx12, workspace=dh)))
        put("swiglu_bwd.unfused", fl, timeit(lambda: (ops.linear_dgrad(dy, w3, out=dh), ops.swiglu_bwd(dh, x12, dx12))))
        put("swiglu_bwd.elementwise_only", fl, timeit(lambda: ops.swiglu_bwd(dh, x12, dx12)))
    out = {}
    for k, v in res.items():
        v = sorted(v)
        tf, us = v[len(v) // 2]
        out[k] = {"tflops": round(tf, 1), "us": round(us, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
