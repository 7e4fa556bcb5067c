"""Data-parallel gradient synchronisation over RCCL (torch.distributed 'nccl' backend on ROCm =
RCCL over xGMI), replacing the DDP reducer that accelerate builds at
src/trainer/common.py:219 (`accelerator.prepare(model)`) and its all-reduce inside
`accelerator.backward` (common.py:376-380), plus the per-step loss gather of
ModelForTraining.log (src/models/for_training.py:171-183).

One bucket per JiT block (7.09 M params for JiT-B/16), one for the final layer and two for the
embeddings / class embedding. Each bucket's all-reduce is launched the moment the engine has
written that bucket's gradients (stream-ordered: RCCL's stream waits on the compute stream at that
point), so communication overlaps the rest of the backward; the fused optimizer then steps each
bucket as soon as its reduction lands (the compute stream waits on that bucket's work only). The
mean over ranks is folded into the optimizer's grad_scale = 1/world (SUM all-reduce, so the same
code runs on gloo in the CPU tests).

Wire dtype. The reference's DDP reduces the parameters' own .grad tensors, which are bf16 (bf16
weights, SURVEY gotcha #5): `wire="bf16"` does the same -- each bucket's f32 gradient is rounded to a
bf16 wire buffer (one HBM pass) and THAT is all-reduced (185 MB + 15 MB class table per JiT-B/16
step, SURVEY §8(e)'s budget); the optimizer reads the reduced bf16 values directly. `wire="f32"`
reduces the f32 gradients (2x the bytes; exact up to summation order).
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
    def __init__(self, grads: torch.Tensor, buckets: list[tuple[str, int, int]], group=None, wire: str = "f32"):
        if wire not in ("f32", "bf16"):
            raise ValueError(f"wire dtype must be 'f32' or 'bf16', got {wire!r}")
        self.grads = grads
        self.buckets = buckets
        self.index = {n: (lo, hi) for n, lo, hi in buckets}
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.wire = wire
        self.comm = torch.empty(grads.numel(), dtype=torch.bfloat16, device=grads.device) \
            if wire == "bf16" and self.world > 1 else None
        self.works: dict[str, object] = {}

    def _to_wire(self, lo: int, hi: int) -> torch.Tensor:
        src, dst = self.grads[lo:hi], self.comm[lo:hi]
        if src.is_cuda:
            from . import ops
            ops.cast_f32_bf16(src, dst)  # HIP kernel on the compute stream (RNE)
        else:
            dst.copy_(src)  # gloo / CPU tensors (tests)
        return dst

    def launch(self, name: str):
        if self.world == 1:
            return
        lo, hi = self.index[name]
        buf = self._to_wire(lo, hi) if self.comm is not None else self.grads[lo:hi]
        self.works[name] = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def launch_rest(self):
        for n, _, _ in self.buckets:
            if n not in self.works:
                self.launch(n)

    def finish(self, apply_fn):
        """For every bucket in completion order: make the current stream wait for its reduction,
        then apply_fn(lo, hi, grad_scale, grad) with grad = the reduced buffer of [lo, hi) (f32 slice of
        the gradient buffer, or the bf16 wire slice)."""
        scale = 1.0 / self.world
        for n, lo, hi in self.buckets:
            w = self.works.pop(n, None)
            if w is not None:
                w.wait()
            src = self.comm[lo:hi] if self.comm is not None else self.grads[lo:hi]
            apply_fn(lo, hi, scale, src)
        self.works.clear()


class LossLog:
    """`accelerator.gather(loss).mean().item()` of ModelForTraining.log (src/models/for_training.py:
    171-183) as ONE async all-reduce of a 2-float [loss_sum, count] tensor per step. The reduced pair is
    copied to pinned host memory behind an event and read `depth - 1` steps later, so the host never
    waits for the step it just enqueued (the reference's per-step gather + .item() is a full sync).
    world 1: no collective."""

    def __init__(self, device, group=None, depth: int = 3):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        dev = torch.device(device)
        self.cuda = dev.type == "cuda"
        self.slots = [torch.zeros(2, dtype=torch.float32, device=dev) for _ in range(depth)]
        self.host = [torch.zeros(2, dtype=torch.float32, pin_memory=self.cuda) for _ in range(depth)]
        self.pending: list[tuple[int, object, object]] = []
        self.k = 0

    def push(self, loss: torch.Tensor) -> float | None:
        """loss: this rank's mean loss (a device scalar); enqueued, not read. Returns the mean over ranks
        of the loss pushed depth-1 calls ago once that many are pending, else None."""
        i = self.k % len(self.slots)
        self.k += 1
        buf = self.slots[i]
        buf[0].copy_(loss.reshape(()))
        buf[1].fill_(1.0)
        work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True) if self.world > 1 else None
        ev = None
        if self.cuda:
            if work is not None:
                work.wait()  # stream-ordered: the current stream waits for the reduction, the host does not
            self.host[i].copy_(buf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self.pending.append((i, work, ev))
        if len(self.pending) >= len(self.slots):
            return self.pop()
        return None

    def pop(self) -> float | None:
        """Mean over ranks of the oldest pushed loss (waits for it only)."""
        if not self.pending:
            return None
        i, work, ev = self.pending.pop(0)
        if ev is not None:
            ev.synchronize()
            s, c = self.host[i].tolist()
        else:
            if work is not None:
                work.wait()
            s, c = self.slots[i].tolist()
        return s / c
