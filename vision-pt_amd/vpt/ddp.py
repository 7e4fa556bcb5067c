"""Data-parallel gradient synchronisation over RCCL (torch.distributed 'nccl' backend on ROCm =
RCCL over xGMI), replacing the DDP reducer that accelerate builds at
src/trainer/common.py:219 (`accelerator.prepare(model)`) and its all-reduce inside
`accelerator.backward` (common.py:376-380).

One bucket per JiT block (7.09 M params = 28 MB of f32 gradient for JiT-B/16), one for the final
layer and two for the embeddings / class embedding. Each bucket's all-reduce is launched the
moment the engine has written that bucket's gradients (stream-ordered: RCCL's stream waits on the
compute stream at that point), so communication overlaps the rest of the backward; the fused
optimizer then steps each bucket as soon as its reduction lands (the compute stream waits on that
bucket's work only). The mean over ranks is folded into the optimizer's grad_scale = 1/world
(SUM all-reduce, so the same code runs on gloo in the CPU tests).
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from .params import ParamLayout


def grad_buckets(layout: ParamLayout, depth: int) -> list[tuple[str, int, int]]:
    """Buckets (name, lo, hi) in the order the backward completes them; they tile [0, total)."""
    by = layout.by_name

    def span(prefix: str):
        ss = [s for s in layout.specs if s.name.startswith(prefix)]
        return min(s.offset for s in ss), max(s.offset + s.numel for s in ss)

    out = []
    f_lo, f_hi = span("final_layer.")
    b_first = span("blocks.0.")[0]
    tail_lo = by["class_encoder.embedding.weight"].offset if "class_encoder.embedding.weight" in by else None
    # final layer bucket extends to the class embedding (or the end): alignment padding included
    out.append(("final", f_lo, tail_lo if tail_lo is not None else layout.total))
    for i in reversed(range(depth)):
        lo = span(f"blocks.{i}.")[0]
        hi = span(f"blocks.{i + 1}.")[0] if i + 1 < depth else f_lo
        out.append((f"block{i}", lo, hi))
    out.append(("embed", 0, b_first))
    if tail_lo is not None:
        out.append(("class_embedding", tail_lo, layout.total))
    return out


class GradSync:
    def __init__(self, grads: torch.Tensor, buckets: list[tuple[str, int, int]], group=None):
        self.grads = grads
        self.buckets = buckets
        self.index = {n: (lo, hi) for n, lo, hi in buckets}
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.works: dict[str, object] = {}

    def launch(self, name: str):
        if self.world == 1:
            return
        lo, hi = self.index[name]
        self.works[name] = dist.all_reduce(self.grads[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def launch_rest(self):
        for n, _, _ in self.buckets:
            if n not in self.works:
                self.launch(n)

    def finish(self, apply_fn):
        """For every bucket in completion order: make the current stream wait for its reduction,
        then apply_fn(lo, hi, grad_scale)."""
        scale = 1.0 / self.world
        for n, lo, hi in self.buckets:
            w = self.works.pop(n, None)
            if w is not None:
                w.wait()
            apply_fn(lo, hi, scale)
        self.works.clear()
