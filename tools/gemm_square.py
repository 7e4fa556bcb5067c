"""Developer microbenchmark: forward GEMM TFLOP/s on square sizes (4096^3, 8192^3) and on the
JiT qkv shape, per forced geometry, with torch.matmul (hipBLASLt) as the known-good bar.
Uniform [-1, 1) operands (guide §5.4 rule 25), interleaved rounds in one process (rule 24).

  python tools/gemm_square.py [--rounds 3]
"""
import os
os.environ.setdefault("VPT_DIAG", "1")  # A/B switches live in libvpt_hip_diag.so only

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


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


GEOS = (256, 2562, 128)


def main():
    global GEOS
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--geos", default="", help="comma list of forced geometries (2563/2564: timing-only ablations)")
    args = ap.parse_args()
    if args.geos:
        GEOS = tuple(int(v) for v in args.geos.split(","))
    shapes = {"4k": (4096, 4096, 4096), "8k": (8192, 8192, 8192), "qkv": (33360, 2304, 768),
              "w3": (33360, 768, 2048), "qkvK4k": (33360, 2304, 4096)}
    res = {}
    for _ in range(args.rounds):
        for name, (M, N, K) in shapes.items():
            x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
            y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            fl = 2.0 * M * N * K
            for geo in GEOS:
                ops.lib.vpt_gemm_set_geometry(geo)
                ms = timeit(lambda: ops.linear(x, w, out=y))
                res.setdefault(f"{name}@{geo}", []).append(fl / (ms * 1e-3) / 1e12)
            ops.lib.vpt_gemm_set_geometry(0)
            ms = timeit(lambda: torch.matmul(x, w.t()))
            res.setdefault(f"{name}@torch", []).append(fl / (ms * 1e-3) / 1e12)
            del x, w, y
    print(json.dumps({k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
