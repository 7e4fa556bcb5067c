"""How a persistent ring GEMM tolerates kernels running beside it (diagnostic library): on a side stream,
`k` one-wave workgroups each hold a CU for T us (vpt_diag_occupy: a stand-in for RCCL's all-reduce channels or the
side-stream optimizer at N > 1), and the GEMM is launched on the main stream right after; its time (HIP events on
the main stream) against k, for the persistent grid (one block per CU, items walked in a fixed stride) and for one
block per item (ring grid = items; the dispatcher places blocks wherever CUs are free).

  python tools/gemm_cobusy_probe.py [--T 150]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=float, default=150.0, help="occupier duration, us")
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    _lib.use_diag()
    lib = _lib.lib
    dev = torch.device("cuda", 0)
    M, D, F = 8 * 4170, 768, 2048
    sink = torch.zeros(64, device=dev)
    x = torch.randn(M, D, device=dev).bfloat16()
    wqkv = (torch.randn(3 * D, D, device=dev) * 0.05).bfloat16()
    dx12 = torch.randn(M, 2 * F, device=dev).bfloat16()
    w12 = (torch.randn(2 * F, D, device=dev) * 0.05).bfloat16()
    yq = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=dev)
    yd = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    gemms = {"qkv_fwd": lambda: ops.linear(x, wqkv, out=yq), "w12_dgrad": lambda: ops.linear_dgrad(dx12, w12, out=yd)}
    main_s, side = torch.cuda.current_stream(), torch.cuda.Stream()
    ticks = int(args.T * 100)
    res = {}
    for mode, rg in (("persistent", 256), ("per_item", 0)):
        lib.vpt_gemm_set_ring_grid(rg)
        for name, fn in gemms.items():
            for k in (0, 8, 32, 128):
                ts = []
                for _ in range(args.reps):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    if k:
                        with torch.cuda.stream(side):
                            lib.vpt_diag_occupy(k, ticks, 96 * 1024, sink.data_ptr(), side.cuda_stream)
                    e0.record(main_s)
                    fn()
                    e1.record(main_s)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                res[f"{mode}/{name}/k{k}"] = round(statistics.median(ts), 1)
                print(mode, name, k, res[f"{mode}/{name}/k{k}"], flush=True)
    lib.vpt_gemm_set_ring_grid(0)
    print(json.dumps({"occupier_us": args.T, "gemm_us": res}))


if __name__ == "__main__":
    main()
