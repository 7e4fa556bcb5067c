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

import contextlib

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
    """Bucketed gradient all-reduce with the optimizer step overlapped (SURVEY §8(e) "Overlap").

    Per step: `arm(apply_fn)` before the backward, `launch(name)` from the engine's on_ready as each bucket's
    last gradient kernel is enqueued, `launch_rest()` after it, `finish()` before the next forward.

    apply_fn(lo, hi, grad_scale, grad, **clip) steps parameters [lo, hi) from `grad` (the reduced f32 slice of
    the gradient buffer or the bf16 wire slice); with clipping configured it also receives clip_coef (device
    f32 scalar) and clip_value (RAdamScheduleFreeFlat.apply_range takes both).

    overlap=True: each bucket is stepped on a side stream the moment its reduction lands (world 1: the
    moment its gradients are written), i.e. during the rest of the backward; finish() joins the side stream
    into the current one (CPU / gloo: the same order, blocking). Safe because a bucket's parameters are never read again in this backward once its
    gradients are complete (the dgrad GEMMs of block i precede on_ready(block i)).

    clip_grad_norm (after_backward, src/models/for_training.py:98-109): the global L2 norm of the mean
    gradient needs every bucket, so landing buckets only contribute partial sums of squares (side stream);
    finish() forms the coefficient on the device (no host sync) and steps every bucket with it.
    clip_grad_value: a clamp inside the optimizer kernel, so it keeps the overlap.

    force_collective=True runs every bucket's all-reduce (and the wire cast) even at world size 1, so the
    collective path -- RCCL's stream-ordered wait inside the side-stream context, the wire cast before it on the
    compute stream -- can be exercised on a one-GPU box (a SUM over one rank is the identity)."""

    def __init__(self, grads: torch.Tensor, buckets: list[tuple[str, int, int]], group=None, wire: str = "f32",
                 overlap: bool = True, clip_grad_norm: float | None = None, clip_grad_value: float | None = None,
                 force_collective: bool = False):
        if wire not in ("f32", "bf16"):
            raise ValueError(f"wire dtype must be 'f32' or 'bf16', got {wire!r}")
        self.grads = grads
        self.buckets = buckets
        self.index = {n: (lo, hi) for n, lo, hi in buckets}
        self.slot = {n: i for i, (n, _, _) in enumerate(buckets)}
        spans = sorted((lo, hi) for _, lo, hi in buckets)
        if any(a[1] != b[0] for a, b in zip(spans, spans[1:])):
            raise ValueError("gradient buckets must tile one contiguous range")
        self.buckets_span = (spans[0][0], spans[-1][1])
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        if force_collective and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("GradSync(force_collective=True) needs an initialised process group")
        self.collective = self.world > 1 or force_collective
        self.wire = wire
        self.cuda = grads.is_cuda
        self.comm = torch.empty(grads.numel(), dtype=torch.bfloat16, device=grads.device) \
            if wire == "bf16" and self.collective else None
        self.overlap = overlap  # land (reduce-wait + step) each bucket as it is launched
        self.side = torch.cuda.Stream(device=grads.device) if (self.cuda and overlap) else None
        self.configure_clipping(clip_grad_norm, clip_grad_value)
        self.works: dict[str, object] = {}
        self.landed: list[str] = []
        self.apply_fn = None
        self.scale = 1.0 / self.world

    def configure_clipping(self, clip_grad_norm: float | None = None, clip_grad_value: float | None = None):
        if clip_grad_norm is not None:
            if clip_grad_norm <= 0:
                raise ValueError("clip_grad_norm must be > 0")
            self.nb = ops_norm_blocks() if self.cuda else 1
            self.part = torch.zeros(len(self.buckets) * self.nb, dtype=torch.float32, device=self.grads.device)
            self.coef = torch.ones(1, dtype=torch.float32, device=self.grads.device)
            self.norm = torch.zeros(1, dtype=torch.float32, device=self.grads.device)  # last step's total norm
        if clip_grad_value is not None and clip_grad_value <= 0:
            raise ValueError("clip_grad_value must be > 0")
        self.clip_norm, self.clip_value = clip_grad_norm, clip_grad_value

    # ------------------------------------------------------------------ per step
    def arm(self, apply_fn, grad_scale: float = 1.0):
        """Registers this step's optimizer callback before the backward (enables the overlap). grad_scale
        multiplies the summed gradient (e.g. 1 / gradient_accumulation_steps); the 1 / world mean is added."""
        self.apply_fn = apply_fn
        self.scale = grad_scale / self.world

    def _src(self, lo: int, hi: int) -> torch.Tensor:
        return self.comm[lo:hi] if self.comm is not None else self.grads[lo:hi]

    def _to_wire(self, lo: int, hi: int) -> torch.Tensor:
        src, dst = self.grads[lo:hi], self.comm[lo:hi]
        if src.is_cuda:
            from . import ops
            ops.cast_f32_bf16(src, dst)  # HIP kernel on the compute stream (RNE)
        else:
            dst.copy_(src)  # gloo / CPU tensors (tests)
        return dst

    def launch(self, name: str):
        if name in self.works or name in self.landed:
            return
        lo, hi = self.index[name]
        if self.collective:
            buf = self._to_wire(lo, hi) if self.comm is not None else self.grads[lo:hi]
            self.works[name] = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            self.works[name] = None
        if self.apply_fn is not None and self.overlap:
            self._land(name)

    def launch_rest(self):
        for n, _, _ in self.buckets:
            self.launch(n)

    def _clip_kw(self) -> dict:
        kw = {}
        if self.clip_norm is not None:
            kw["clip_coef"] = self.coef
        if self.clip_value is not None:
            kw["clip_value"] = self.clip_value
        return kw

    def _sumsq(self, name: str, src: torch.Tensor, scale: float):
        i = self.slot[name]
        part = self.part[i * self.nb:(i + 1) * self.nb]
        if src.is_cuda:
            from . import ops
            ops.grad_sumsq(src, scale, part)
        else:
            part.copy_((src.float() * scale).pow(2).sum().reshape(1))

    def _land(self, name: str):
        """The bucket's reduction has been enqueued: step it (or, with global-norm clipping, take its sum of
        squares) behind that reduction -- on the side stream when overlapping, else on the current stream."""
        w = self.works.pop(name)
        lo, hi = self.index[name]
        scale = self.scale
        src = self._src(lo, hi)
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream(self.grads.device))  # gradients / wire cast written
            ctx = torch.cuda.stream(self.side)
        else:
            ctx = contextlib.nullcontext()
        with ctx:
            if w is not None:
                w.wait()  # stream-ordered on the GPU (the side / current stream waits the collective); blocking on gloo
            if self.clip_norm is not None:
                self._sumsq(name, src, scale)
            else:
                self.apply_fn(lo, hi, scale, src, **self._clip_kw())
        self.landed.append(name)

    def finish(self, apply_fn=None, grad_scale: float = 1.0):
        """Completes the step: every bucket not yet landed is landed now (serial path), global-norm clipping
        forms its coefficient and steps every bucket, and the current stream waits for the side stream.
        `apply_fn` (if given) replaces the armed callback -- the serial form finish(fn) without arm()."""
        if apply_fn is not None:
            self.apply_fn = apply_fn
            self.scale = grad_scale / self.world
        if self.apply_fn is None:
            raise RuntimeError("GradSync.finish: no optimizer callback (arm() or finish(apply_fn))")
        if not self.collective and not self.overlap and self.clip_norm is None and not self.landed:
            # one process, serial: the buckets tile the flat buffer, so ONE optimizer launch covers them all
            lo, hi = self.buckets_span
            self.apply_fn(lo, hi, self.scale, self.grads[lo:hi], **self._clip_kw())
            self.works.clear()
            self.apply_fn = None
            return
        for n, _, _ in self.buckets:
            if n not in self.landed and n not in self.works:
                self.launch(n)  # (lands it as well when overlapping)
        for n, _, _ in self.buckets:
            if n in self.works:
                self._land(n)
        if self.clip_norm is not None:
            ctx = torch.cuda.stream(self.side) if self.side is not None else contextlib.nullcontext()
            scale = self.scale
            with ctx:
                if self.part.is_cuda:
                    from . import ops
                    ops.clip_coef(self.part, self.clip_norm, self.coef, self.norm)
                else:
                    self.norm.copy_(self.part.sum().sqrt().reshape(1))
                    self.coef.copy_((self.clip_norm / (self.norm + 1e-6)).clamp(max=1.0))
                for n, lo, hi in self.buckets:
                    self.apply_fn(lo, hi, scale, self._src(lo, hi), **self._clip_kw())
        if self.side is not None:
            torch.cuda.current_stream(self.grads.device).wait_stream(self.side)
        self.works.clear()
        self.landed = []
        self.apply_fn = None


def ops_norm_blocks() -> int:
    from . import ops
    return ops.grad_norm_blocks()


class LossLog:
    """`accelerator.gather(loss).mean().item()` of ModelForTraining.log (src/models/for_training.py:
    171-183) as ONE async all-reduce of a 2-float [loss_sum, count] tensor per step. The reduced pair is
    copied to pinned host memory behind an event and read `depth - 1` steps later, so the host never
    waits for the step it just enqueued (the reference's per-step gather + .item() is a full sync).
    world 1: no collective (force_collective=True: the all-reduce anyway, as GradSync's)."""

    def __init__(self, device, group=None, depth: int = 3, force_collective: bool = False):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.collective = self.world > 1 or force_collective
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
        work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True) if self.collective else None
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
