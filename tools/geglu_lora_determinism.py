"""Repeated vpt_geglu_bwd_lora / vpt_geglu_fwd_lora launches on the same inputs: rows whose vs / ds differ from the
first launch (and unwritten rows), per launch.

  python tools/geglu_lora_determinism.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def main():
    dev = "cuda"
    torch.manual_seed(0)
    for M, F in ((4100, 5120), (4224, 5120), (333, 2560)):
        dy = torch.randn(M, F, device=dev).bfloat16()
        x12 = torch.randn(M, 2 * F, device=dev).bfloat16()
        up = (torch.randn(2 * F, 16, device=dev) * 0.05).bfloat16()
        down = (torch.randn(16, F, device=dev) * 0.05).bfloat16()
        for kind in ("bwd", "fwd"):
            outs = []
            for _ in range(8):
                v = torch.full((M, 16), float("nan"), dtype=torch.bfloat16, device=dev)
                if kind == "bwd":
                    ops.geglu_bwd_lora(dy, x12, up, 0.0625, v)
                else:
                    ops.geglu_fwd_lora(x12, down, 0.0625, v)
                outs.append(v)
            torch.cuda.synchronize()
            ref = (dy.float() if kind == "bwd" else None)
            rep = []
            for v in outs:
                nan_rows = int(torch.isnan(v.float()).any(1).sum())
                diff = (v.view(torch.int16) != outs[0].view(torch.int16)).any(1)
                rows = diff.nonzero().flatten().tolist()
                rep.append((nan_rows, len(rows), rows[:6]))
            print(kind, M, F, rep, flush=True)


if __name__ == "__main__":
    main()
