"""Where the SwiGLU-backward dgrad ring GEMM's time goes (dh = dY . W3 with the SwiGLU backward in the epilogue,
x12 read and dx12 written there; denoiser.py:480-506 backward): time per call against M at the C3 shapes' row-tile
counts (items = row tiles x 8 on 256 CUs, so 128 row tiles = 4 full rounds; M = 32848 / 33232 are 129 / 130 row tiles),
with the production epilogue and its timing ablations (diagnostic library, wrong results: no epilogue, dx12 stores
dropped, x12 read from one L2-resident tile), plus the plain bf16-output GEMM of the same shape with and without its
epilogue.

  python tools/swb_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402


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
    _lib.use_diag()
    dev = "cuda"
    D, F = 768, 2048
    Mmax = 136 * 256
    dy = torch.randn(Mmax, D, device=dev).bfloat16()
    w3 = (torch.randn(D, F, device=dev) * 0.05).bfloat16()
    x12 = torch.randn(Mmax, 2 * F, device=dev).bfloat16()
    dx12 = torch.empty(Mmax, 2 * F, dtype=torch.bfloat16, device=dev)
    dh = torch.empty(Mmax, F, dtype=torch.bfloat16, device=dev)
    res = {}
    for M in [120 * 256, 124 * 256, 127 * 256, 128 * 256, 32848, 33232, 131 * 256, 132 * 256, 136 * 256]:
        row = {}
        for abl, tag in ((0, "prod"), (3, "no_epi"), (4, "no_store"), (6, "x12_l2")):
            _lib.lib.vpt_gemm_set_swb_ablation(abl)
            row[f"swb_{tag}"] = round(timeit(lambda: ops.linear_dgrad_swiglu(dy[:M], w3, x12[:M], dx12[:M],
                                                                             workspace=dh[:M])), 2)
        _lib.lib.vpt_gemm_set_swb_ablation(0)
        row["plain_bf16_out"] = round(timeit(lambda: ops.linear_dgrad(dy[:M], w3, out=dh[:M])), 2)
        _lib.lib.vpt_gemm_set_geometry(2568)
        row["plain_no_epi"] = round(timeit(lambda: ops.linear_dgrad(dy[:M], w3, out=dh[:M])), 2)
        _lib.lib.vpt_gemm_set_geometry(0)
        res[M] = row
        print(M, json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
