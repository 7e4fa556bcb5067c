"""The C3 step's HBM-bound pixel kernels alone (B=8, 1024^2 fp16 images): patchify with the in-kernel noise, with an
explicit fp16 noise tensor, and without noising; the flow loss (image and velocity targets). HIP events on the
launching stream, median per launch; GB/s from the algorithmic bytes (fp16 pixel in + bf16 patch out,
+2 B/px for explicit noise; loss: bf16 prediction + fp16 image in, bf16 gradient out). `--lib NAME` runs a variant
build (lib/var/libvpt_hip_NAME.so).

  python tools/hbm_kernels.py [--lib NAME]
"""
import argparse
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
    cases = {
        "patchify_gen_noise": (lambda: ops.patchify(img, B, H, W, out, t=t, seed=5), 4.0 * n),
        "patchify_explicit_noise": (lambda: ops.patchify(img, B, H, W, out, t=t, noise=noise), 6.0 * n),
        "patchify_copy": (lambda: ops.patchify(img, B, H, W, out, noising=False), 4.0 * n),
        "flow_loss_image": (lambda: ops.flow_loss(pred, img, t, B, H, W, dpred, part, loss, target=0), 6.0 * n),
        "flow_loss_velocity_gen": (lambda: ops.flow_loss(pred, img, t, B, H, W, dpred, part, loss, target=1, seed=5),
                                   6.0 * n),
    }
    res = {}
    for name, (fn, nbytes) in cases.items():
        us = statistics.median(timeit(fn) for _ in range(3))
        gbs = nbytes / us / 1e3
        res[name] = {"us": round(us, 2), "gb_s": round(gbs, 1), "frac_of_8TBs": round(gbs / PEAK, 3)}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps({"lib": args.lib, "shape": [B, 3, H, W], "kernels": res}))


if __name__ == "__main__":
    main()
