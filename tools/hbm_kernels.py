"""The C3 step's HBM-bound pixel kernels alone (B=8, 1024^2 fp16 images): patchify with the in-kernel noise, with an
explicit fp16 noise tensor, and without noising; the flow loss (image and velocity targets). HIP events on the
launching stream, median per launch; GB/s from the algorithmic bytes (fp16 pixel in + bf16 patch out,
+2 B/px for explicit noise; loss: bf16 prediction + fp16 image in, bf16 gradient out); and the QK-norm + RoPE backward at
the C3 shape (M = 8 x 4154 token rows, D = 768: dq | dk and q | k in, dq | dk out) and the RMSNorm forward there. `--lib NAME` runs a variant build
(lib/var/libvpt_hip_NAME.so); each case's output digest (sha1 of its bytes) is printed for bitwise comparisons.

  python tools/hbm_kernels.py [--lib NAME]
"""
import argparse
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402

PEAK = 8000.0  # GB/s


def timeit(fn, iters=20):
    fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    ev[0].record()
    for i in range(iters):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    return statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(iters)) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    if args.lib:
        from vpt._build import PKG_ROOT
        _lib.use_library(PKG_ROOT / "lib" / "var" / f"libvpt_hip_{args.lib}.so")
    dev = "cuda"
    B, H, W = 8, 1024, 1024
    n = B * 3 * H * W
    g = torch.Generator(device=dev).manual_seed(0)
    img = (torch.rand(B, 3, H, W, device=dev, generator=g) * 2 - 1).half()
    noise = torch.randn(B, 3, H, W, device=dev, generator=g).half()
    t = torch.rand(B, device=dev, generator=g)
    npch = B * (H // 16) * (W // 16)
    out = torch.empty(npch, 768, dtype=torch.bfloat16, device=dev)
    pred = torch.randn(npch, 768, device=dev, generator=g).bfloat16()
    dpred = torch.empty_like(pred)
    part = torch.empty(ops.loss_blocks(), device=dev)
    loss = torch.empty(1, device=dev)
    rps = 4154
    M = B * rps
    D = 768
    qkv = torch.randn(M, 3 * D, device=dev, generator=g).bfloat16()
    dqk = torch.randn(M, 2 * D, device=dev, generator=g).bfloat16()
    wq = (1 + 0.1 * torch.randn(64, device=dev, generator=g)).bfloat16()
    wk = (1 + 0.1 * torch.randn(64, device=dev, generator=g)).bfloat16()
    ang = torch.rand(rps, 32, device=dev, generator=g) * 6.28
    cos_t, sin_t = ang.cos().contiguous(), ang.sin().contiguous()
    dqkv = torch.zeros(M, 3 * D, dtype=torch.bfloat16, device=dev)
    dwp = torch.empty(ops.qknorm_rope_blocks(M), 128, device=dev)
    xr = torch.randn(M, D, device=dev, generator=g).bfloat16()
    wr = (1 + 0.1 * torch.randn(D, device=dev, generator=g)).bfloat16()
    yr = torch.empty_like(xr)
    rs = torch.empty(M, device=dev)
    outs = {"rmsnorm_fwd_c3": yr, "patchify_gen_noise": out, "patchify_explicit_noise": out, "patchify_copy": out,
            "flow_loss_image": dpred, "flow_loss_velocity_gen": dpred, "qknorm_rope_bwd_c3": dqkv}
    cases = {
        "patchify_gen_noise": (lambda: ops.patchify(img, B, H, W, out, t=t, seed=5), 4.0 * n),
        "patchify_explicit_noise": (lambda: ops.patchify(img, B, H, W, out, t=t, noise=noise), 6.0 * n),
        "patchify_copy": (lambda: ops.patchify(img, B, H, W, out, noising=False), 4.0 * n),
        "flow_loss_image": (lambda: ops.flow_loss(pred, img, t, B, H, W, dpred, part, loss, target=0), 6.0 * n),
        "flow_loss_velocity_gen": (lambda: ops.flow_loss(pred, img, t, B, H, W, dpred, part, loss, target=1, seed=5),
                                   6.0 * n),
        "rmsnorm_fwd_c3": (lambda: ops.rmsnorm_fwd(xr, wr, yr, rs), 4.0 * M * D + 4.0 * M),
        "qknorm_rope_bwd_c3": (lambda: ops.qknorm_rope_bwd(dqk, qkv, wq, wk, cos_t, sin_t, rps, dqkv, dwp), 12.0 * M * D),
    }
    res = {}
    for name, (fn, nbytes) in cases.items():
        us = statistics.median(timeit(fn) for _ in range(3))
        gbs = nbytes / us / 1e3
        torch.cuda.synchronize()
        digest = hashlib.sha1(outs[name].view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12]
        res[name] = {"us": round(us, 2), "gb_s": round(gbs, 1), "frac_of_8TBs": round(gbs / PEAK, 3), "sha1": digest}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps({"lib": args.lib, "shape": [B, 3, H, W], "kernels": res}))


if __name__ == "__main__":
    main()
