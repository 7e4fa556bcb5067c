"""Timeline diagnostic of the persistent 256x256 ring GEMM (geometry 2567): per block, s_memrealtime
(100 MHz) stamps of each item's start, tile-0-ready, K-loop end and epilogue end. Prints medians of
the phases and the dispatch skew, in microseconds, per shape, plus the kernel's event-timed duration.

  python tools/gemm_timeline.py
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


def med(t):
    t = t.flatten()
    return round(t.median().item(), 2) if t.numel() else None


def main():
    dbg = torch.zeros(256 * 4 * 4 + 64, dtype=torch.int64, device="cuda")
    ops.lib.vpt_gemm_set_debug(dbg.data_ptr())
    out = {}
    for name, (M, N, K) in {"1round_k256": (16384, 1024, 256), "1round_k768": (16384, 1024, 768),
                            "o_k768": (33360, 768, 768), "qkv_k768": (33360, 2304, 768),
                            "w3_k2048": (33360, 768, 2048)}.items():
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        ops.lib.vpt_gemm_set_geometry(2567)
        for _ in range(3):
            ops.linear(x, w, out=y)
        dbg.zero_()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.linear(x, w, out=y)
        e.record()
        torch.cuda.synchronize()
        ops.lib.vpt_gemm_set_geometry(0)
        d = dbg[:256 * 16].view(256, 4, 4).double().cpu()
        used = d[:, :, 0] > 0
        t0 = d[:, 0, 0][used[:, 0]].min()
        us = (d - t0) / 100.0  # 100 MHz -> us
        ph = {}
        ph["event_us"] = round(s.elapsed_time(e) * 1e3, 1)
        ph["span_us"] = round((us[:, :, 3][used].max()).item(), 1)
        ph["start_skew_us"] = med(us[:, 0, 0][used[:, 0]])
        ph["start_max_us"] = round(us[:, 0, 0][used[:, 0]].max().item(), 2)
        for k in range(4):
            m = used[:, k]
            if not m.any():
                break
            ph[f"item{k}"] = {"n": int(m.sum()), "start": med(us[:, k, 0][m]), "wait_tile0": med((us[:, k, 1] - us[:, k, 0])[m]),
                              "kloop": med((us[:, k, 2] - us[:, k, 1])[m]), "epilogue": med((us[:, k, 3] - us[:, k, 2])[m]),
                              "end": med(us[:, k, 3][m])}
        out[name] = ph
        del x, w, y
    ops.lib.vpt_gemm_set_debug(None)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
