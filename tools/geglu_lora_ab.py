"""In-process A/B of vpt_geglu_bwd_lora between builds of the library (vpt._build.build_variant: lib/var/
libvpt_hip_<name>.so; "base" = lib/libvpt_hip.so) at config 5's shapes; HIP-event medians per launch, interleaved.

  python tools/geglu_lora_ab.py --variants base,gbabl1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402
from vpt._build import LIB, PKG_ROOT  # noqa: E402


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    libs = {v: _lib.load_library(LIB if v == "base" else PKG_ROOT / "lib" / "var" / f"libvpt_hip_{v}.so")
            for v in args.variants.split(",")}
    dev = "cuda"
    res = {}
    for M, F in ((4224, 5120), (4096, 5120), (16896, 2560)):
        dy = torch.randn(M, F, device=dev).bfloat16()
        x12 = torch.randn(M, 2 * F, device=dev).bfloat16()
        up = (torch.randn(2 * F, 16, device=dev) * 0.05).bfloat16()
        vs = torch.empty(M, 16, dtype=torch.bfloat16, device=dev)
        down = (torch.randn(16, F, device=dev) * 0.05).bfloat16()
        gg = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
        cases = {"bwd_lora": lambda: ops.geglu_bwd_lora(dy, x12, up, 0.0625, vs),
                 "fwd_lora": lambda: ops.geglu_fwd_lora(x12, down, 0.0625, vs, out=gg),
                 "fwd+lora_proj": lambda: (ops.geglu_fwd(x12, out=gg), ops.lora_proj(gg, down, True, vs, alpha=0.0625))}
        t = {(v, c): [] for v in libs for c in cases}
        for _ in range(args.rounds):
            for v, lb in libs.items():
                _lib.use_library(lb)
                for c, fn in cases.items():
                    t[(v, c)].append(timeit(fn))
        outs = {}
        for v, lb in libs.items():  # each build's outputs, compared bitwise with the first build's
            _lib.use_library(lb)
            vb, vf = torch.empty_like(vs), torch.empty_like(vs)
            dx = ops.geglu_bwd_lora(dy, x12, up, 0.0625, vb)
            gf = ops.geglu_fwd_lora(x12, down, 0.0625, vf)
            torch.cuda.synchronize()
            outs[v] = (vb, vf, dx, gf)
        _lib.use_library(libs[next(iter(libs))])
        res[f"{M}x{F}"] = {f"{v}:{c}": round(sorted(x)[len(x) // 2], 1) for (v, c), x in t.items()}
        first = outs[next(iter(outs))]
        res[f"{M}x{F}"]["bitwise_equal"] = {v: all(torch.equal(a, b) for a, b in zip(o, first)) for v, o in outs.items()}
        print(json.dumps({f"{M}x{F}": res[f"{M}x{F}"]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
