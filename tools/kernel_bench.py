"""Developer microbenchmark: per-shape TFLOP/s of the HIP GEMM (fwd / dgrad / wgrad) and attention
kernels at the JiT-B/16 1024^2 B=8 shapes, with torch.matmul (hipBLASLt) timed beside the GEMMs as a
known-good reference bar. Interleaved rounds in one process (guide §5.4 rule 24), random data.

  python tools/kernel_bench.py [--rounds 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402

_lib.use_diag()  # A/B switches live in libvpt_hip_diag.so only


def timeit(fn, iters=10):
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
    ap.add_argument("--attn-only", action="store_true")
    args = ap.parse_args()
    dev = "cuda"
    M = args.M
    shapes = {"qkv": (2304, 768), "o": (768, 768), "w12": (4096, 768), "w3": (768, 2048)}
    res = {}
    ws = torch.empty(64 * 4096 * 2048, dtype=torch.float32, device=dev)
    for r in range(args.rounds):
        for name, (N, K) in ({} if args.attn_only else shapes).items():
            x = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
            dy = (torch.randn(M, N, device=dev) * 0.5).bfloat16()
            y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
            dw = torch.empty(N, K, dtype=torch.float32, device=dev)
            fl = 2.0 * M * N * K
            sp = ops.wgrad_splits(N, K, M)
            t = {}
            for geo in (0, 128, 256, 2561, 2562):
                _lib.lib.vpt_gemm_set_geometry(geo)
                sfx = {0: "", 128: "@128", 256: "@256pp", 2561: "@256ring", 2562: "@256_2stage"}[geo]
                t["fwd" + sfx] = timeit(lambda: ops.linear(x, w, out=y))
                t["dgrad" + sfx] = timeit(lambda: ops.linear_dgrad(dy, w, out=dx))
                t["wgrad" + sfx] = timeit(lambda: ops.linear_wgrad(dy, x, dw, splits=sp, workspace=ws))
            _lib.lib.vpt_gemm_set_geometry(0)
            t.update({
                "torch_fwd": timeit(lambda: torch.matmul(x, w.t())),
                "torch_dgrad": timeit(lambda: torch.matmul(dy, w)),
                "torch_wgrad": timeit(lambda: torch.matmul(dy.t(), x)),
            })
            for k, ms in t.items():
                res.setdefault(f"{name}.{k}", []).append(fl / (ms * 1e-3) / 1e12)
        # attention at the 1024x1024 bucket
        B, H, n = 8, 12, 4170
        rows = n
        qkv = (torch.randn(B * rows, 3 * 768, device=dev)).bfloat16()
        o = torch.empty(B * rows, 768, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B, H, rows, device=dev)
        delta = torch.empty_like(lse)
        do = torch.randn(B * rows, 768, device=dev).bfloat16()
        dq, dk, dv = (torch.empty(B * rows, 768, dtype=torch.bfloat16, device=dev) for _ in range(3))
        q4, k4, v4 = (ops._t4(qkv, B, rows, H, c) for c in (0, 768, 1536))
        o4 = ops._t4(o, B, rows, H)
        fl = 4.0 * B * H * n * n * 64
        tf = timeit(lambda: ops.attn_fwd(q4, k4, v4, o4, lse, None, B, H, rows, n, n))
        tb = timeit(lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, None,
                                         ops._t4(dq, B, rows, H), ops._t4(dk, B, rows, H), ops._t4(dv, B, rows, H),
                                         B, H, rows, n, n))
        for var in (1, 2, 4, 5, 6, 7, 8):  # timing-only ablations of the backward (wrong results)
            _lib.lib.vpt_attn_set_variant(var)
            tv = timeit(lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, None,
                                             ops._t4(dq, B, rows, H), ops._t4(dk, B, rows, H),
                                             ops._t4(dv, B, rows, H), B, H, rows, n, n))
            _lib.lib.vpt_attn_set_variant(0)
            res.setdefault(f"attn.bwd_alg_abl{var}", []).append(2 * fl / (tv * 1e-3) / 1e12)
            res.setdefault(f"attn.bwd_ms_abl{var}", []).append(tv)
        _lib.lib.vpt_attn_set_variant(3)  # 8-wave blocks (A/B)
        tf4 = timeit(lambda: ops.attn_fwd(q4, k4, v4, o4, lse, None, B, H, rows, n, n))
        tb4 = timeit(lambda: ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, None,
                                          ops._t4(dq, B, rows, H), ops._t4(dk, B, rows, H), ops._t4(dv, B, rows, H),
                                          B, H, rows, n, n))
        _lib.lib.vpt_attn_set_variant(0)
        res.setdefault("attn.fwd_8wave", []).append(fl / (tf4 * 1e-3) / 1e12)
        res.setdefault("attn.bwd_alg_8wave", []).append(2 * fl / (tb4 * 1e-3) / 1e12)
        res.setdefault("attn.fwd", []).append(fl / (tf * 1e-3) / 1e12)
        res.setdefault("attn.bwd_alg", []).append(2 * fl / (tb * 1e-3) / 1e12)
        res.setdefault("attn.fwd_ms", []).append(tf)
        res.setdefault("attn.bwd_ms", []).append(tb)
        qh = qkv[:, :768].view(B, rows, H, 64).transpose(1, 2)
        kh = qkv[:, 768:1536].view(B, rows, H, 64).transpose(1, 2)
        vh = qkv[:, 1536:].view(B, rows, H, 64).transpose(1, 2)
        try:
            ts = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qh, kh, vh), iters=5)
            res.setdefault("attn.torch_sdpa_nomask", []).append(fl / (ts * 1e-3) / 1e12)
        except Exception as ex:  # noqa: BLE001
            res["attn.torch_sdpa_nomask"] = [str(ex)[:80]]
    out = {k: (round(sorted(v)[len(v) // 2], 1) if isinstance(v[0], float) else v[0]) for k, v in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
