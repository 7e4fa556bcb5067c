"""Stamp diagnostic of the 256x256 ring GEMM (geometry 2566): where a K step spends its cycles.
Shares only -- the stamps' lgkmcnt(0) waits forbid overlaps of the real kernel (guide §7 In-kernel stamps).

  python tools/gemm_stamp.py
"""
import os
os.environ.setdefault("VPT_DIAG", "1")  # A/B switches live in libvpt_hip_diag.so only

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402

SEGS = ["dma_issue", "ds_reads", "vmcnt_wait", "barrier_Y", "mfma_issue", "barrier_X"]


def main():
    dbg = torch.zeros(256 * 8 * 8, dtype=torch.int64, device="cuda")
    ops.lib.vpt_gemm_set_debug(dbg.data_ptr())
    out = {}
    for name, (M, N, K) in {"qkv": (33360, 2304, 768), "8k": (8192, 8192, 8192), "4k": (4096, 4096, 4096)}.items():
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ops.lib.vpt_gemm_set_geometry(2566)
        dbg.zero_()
        ops.linear(x, w, out=y)
        torch.cuda.synchronize()
        ops.lib.vpt_gemm_set_geometry(0)
        d = dbg.view(256, 8, 8).double().cpu()
        nk = d[:, :, 6]
        valid = nk > 0
        per = {}
        for i, sname in enumerate(SEGS):
            v = (d[:, :, i][valid] / nk[valid])
            per[sname] = round(v.mean().item(), 1)
        tot = sum(per.values())
        per["total_cycles_per_kstep"] = round(tot, 1)
        per["shares"] = {k: round(per[k] / tot, 3) for k in SEGS}
        wg = d[:, :, :6].sum(-1)[valid] / nk[valid]
        per["wave0_vs_wave4"] = [round((d[:, 0, :6].sum(-1) / nk[:, 0].clamp_min(1)).mean().item(), 1),
                                 round((d[:, 4, :6].sum(-1) / nk[:, 4].clamp_min(1)).mean().item(), 1)]
        out[name] = per
        del x, w, y
    ops.lib.vpt_gemm_set_debug(None)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
