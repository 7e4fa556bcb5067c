"""Same-process A/B of attention forward variants (diagnostic library, VPT_DIAG=1): median ms per forward launch
at the bench shape (B=8, H=12, n=4170, 64 context keys) for each vpt_attn_set_rows64 mask, interleaved rounds, and
a bitwise comparison of every variant's o / lse with the first one's.
  VPT_DIAG=1 python tools/attn_fwd_ab.py 0 256"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
import torch  # noqa: E402

from vpt import ops  # noqa: E402


def main():
    masks = [int(a) for a in sys.argv[1:]] or [0, 256]
    dev = "cuda"
    B, H, n = 8, 12, 4170
    rows, D = n, 768
    n_dense = n - 64
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * rows, 3 * D, device=dev, generator=g).bfloat16()
    qkv[:, :D] = (qkv[:, :D].float() * ops.attn_q_scale(0.125)).bfloat16()
    kb = torch.zeros(B, rows, device=dev)
    for b in range(B):
        kb[b, n_dense + 8 + 7 * b:] = float("-inf")
    q4, k4, v4 = (ops._t4(qkv, B, rows, H, c) for c in (0, D, 2 * D))
    outs = {m: (torch.empty(B * rows, D, dtype=torch.bfloat16, device=dev), torch.empty(B, H, rows, device=dev))
            for m in masks}

    def fwd(m):
        o, lse = outs[m]
        ops.lib.vpt_attn_set_rows64(m)
        ops.attn_fwd(q4, k4, v4, ops._t4(o, B, rows, H), lse, kb, B, H, rows, n, n_dense)

    times = {m: [] for m in masks}
    for _ in range(7):
        for m in masks:
            fwd(m)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                fwd(m)
            e.record()
            torch.cuda.synchronize()
            times[m].append(s.elapsed_time(e) / 20)
    ops.lib.vpt_attn_set_rows64(0)
    ref = outs[masks[0]]
    res = {str(m): {"ms": round(statistics.median(times[m]), 4),
                    "bitwise_equal_to_first": all(torch.equal(a, b) for a, b in zip(outs[m], ref))} for m in masks}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
