"""Throughput of the bucketed-batch transform (decoded uint8 -> fp16 bucket crop): the HIP path
(vpt_cover_resize_crop, image already in HBM) beside the reference's CPU chain (oracle/data_oracle.py:
fp16 normalise + ATen antialiased bicubic + crop) on the host threads. Prints one JSON line.

  python tools/data_bench.py [--n 32]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    args = ap.parse_args()
    from vpt import data as D
    from oracle import data_oracle as DO

    H, W, tw, th = 1536, 2048, 1152, 896   # a 3 MP photo into the 1152x896 bucket (1.33x downscale)
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    sw, sh = D.cover_size(W, H, tw, th)
    top, left = D.crop_params(sw, sh, tw, th, torch.Generator().manual_seed(0))
    dimg = torch.from_numpy(img).cuda()
    out = torch.empty(args.n, 3, th, tw, dtype=torch.float16, device="cuda")
    from vpt import ops
    ws = torch.empty(ops.cover_resize_crop_workspace(H, W, sh, sw, top, th, tw) // 4 + 1, dtype=torch.float32,
                     device="cuda")
    for i in range(3):
        D.cover_resize_crop(dimg, tw, th, out[i], top, left, (sw, sh), ws)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(args.n):
        D.cover_resize_crop(dimg, tw, th, out[i], top, left, (sw, sh), ws)
    e.record()
    torch.cuda.synchronize()
    gpu_ms = s.elapsed_time(e) / args.n
    # bytes: uint8 image read (rows the crop needs) + fp16 crop written
    gb = (H * W * 3 + 3 * th * tw * 2) / 1e9
    t0 = time.perf_counter()
    n_cpu = 0
    while time.perf_counter() - t0 < 10.0 and n_cpu < 16:
        DO.transform_chain(img, tw, th, top, left)
        n_cpu += 1
    cpu_s = (time.perf_counter() - t0) / n_cpu
    print(json.dumps({"metric": "bucketed image transform (uint8 HxWx3 -> fp16 bucket crop)",
                      "shape": f"{W}x{H} -> {tw}x{th}", "gpu_ms_per_image": round(gpu_ms, 4),
                      "gpu_images_per_s": round(1e3 / gpu_ms, 1), "gpu_GBps_compulsory": round(gb / (gpu_ms * 1e-3), 1),
                      "cpu_images_per_s": round(1.0 / cpu_s, 2), "cpu_threads": torch.get_num_threads(),
                      "cpu_kind": "port (oracle/data_oracle.py: torch CPU interpolate)"}))


if __name__ == "__main__":
    main()
