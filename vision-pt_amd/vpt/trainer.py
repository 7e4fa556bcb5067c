"""The training loop around the fused JiT step: the reference's Trainer.training_loop /
backward / apply_gradients (src/trainer/common.py:308-388) with its optimizer train()/eval() toggles
(:276-285), gradient accumulation, EMA copy (:211-216, :385-386), saving strategy and callbacks
(src/saving/util.py ModelSavingStrategy, `{name}_{epoch:05}e_{steps:06}s.safetensors`, `ema_` prefix,
common.py:150-164, :390-420) and per-step loss logging (for_training.py:171-189).

What is not here (outside SURVEY §8): previews, W&B / HF-Hub callbacks, eval dataloaders, the accelerate
object. The step itself is vpt.jit_train.JiTTrainer.step (one HIP schedule), the optimizer
vpt.optim.RAdamScheduleFreeFlat, the DDP reducer vpt.ddp.GradSync.
"""

from __future__ import annotations

import os
from typing import Iterable

import torch
import torch.distributed as dist
from safetensors.torch import save_file

from . import ops
from .checkpoint import CLASS_KEY
from .jit_train import ClassTokenizer, JiTTrainer
from .optim import RAdamScheduleFreeFlat


class SavingStrategy:
    """ModelSavingStrategy (src/saving/util.py:15-120): per_epochs (int, or float < 1 = a fraction of an
    epoch in steps), per_steps, save_last; same sanity checks and should_save(epoch, steps) decisions."""

    def __init__(self, total_epochs: int, steps_per_epoch: int, per_epochs: int | float | None = 1,
                 per_steps: int | None = None, save_last: bool = True):
        self.per_epochs, self.per_steps, self.save_last = per_epochs, per_steps, save_last
        self._total_epochs, self._steps_per_epoch = total_epochs, steps_per_epoch
        self._check()

    def _check(self):
        if self.per_epochs is None and self.per_steps is None:
            return
        if self.per_epochs is not None:
            if self.per_epochs <= 0:
                raise ValueError("per_epochs must be greater than 0")
            if isinstance(self.per_epochs, float):
                if self.per_epochs >= 1:
                    raise ValueError("per_epochs must be less than 1 if float")
                if self.per_steps is not None:
                    raise ValueError("per_epochs and per_steps cannot be set together")
            elif self.per_epochs > self._total_epochs:
                raise ValueError("per_epochs must be less than or equal to total_epochs")
        if self.per_steps is not None:
            if self.per_steps <= 0:
                raise ValueError("per_steps must be greater than 0")
            if self.per_steps > self._total_epochs * self._steps_per_epoch:
                raise ValueError("per_steps must be less than or equal to total_steps")

    @property
    def _per_steps(self) -> int | None:
        if isinstance(self.per_epochs, float):
            return int(self.per_epochs * self._steps_per_epoch)
        return self.per_steps

    def should_save(self, epoch: int, steps: int) -> bool:
        if self._steps_per_epoch is None and self._total_epochs is None:
            return False
        if epoch == 0 and steps == 0:
            return False
        if self.per_epochs is not None and epoch != 0:
            if steps % (self._steps_per_epoch * self.per_epochs) == 0:
                return True
        if self._per_steps is not None and steps != 0:
            if steps % self._per_steps == 0:
                return True
        return False


class SafetensorsSaver:
    """SafetensorsSavingCallback (src/saving/safetensors.py:14-35): `save_dir / template.format(name, epoch,
    steps)` with the JiTModel state-dict keys (`denoiser.*`, `class_encoder.embedding.weight`)."""

    template = "{name}_{epoch:05}e_{steps:06}s.safetensors"

    def __init__(self, name: str, save_dir: str, template: str | None = None):
        self.name, self.save_dir = name, save_dir
        if template is not None:
            self.template = template

    def save(self, state_dict: dict[str, torch.Tensor], epoch: int, steps: int, metadata: dict | None = None) -> str:
        path = os.path.join(self.save_dir, self.template.format(name=self.name, epoch=epoch, steps=steps))
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        save_file({k: v.detach().cpu().contiguous() for k, v in state_dict.items()}, path, metadata)
        return path


class ParamEMA:
    """AveragedModel(get_ema_avg_fn(decay), use_buffers=False) over the flat bf16 parameter buffer: one fused
    kernel per update (vpt_ema_update), first update copies (n_averaged == 0)."""

    def __init__(self, params: torch.Tensor, decay: float = 0.9999):
        self.params, self.decay = params, decay
        self.ema = torch.empty_like(params)
        self.n_averaged = 0

    @torch.no_grad()
    def update(self):
        ops.ema_update(self.ema, self.params, self.decay, self.n_averaged == 0)
        self.n_averaged += 1


def reference_state_dict(trainer: JiTTrainer, flat: torch.Tensor | None = None) -> dict[str, torch.Tensor]:
    """JiTModel keys over the engine's layout; `flat` selects another buffer of the same layout (EMA)."""
    eng = trainer.engine
    src = eng.params if flat is None else flat
    out = {}
    for s in eng.layout.specs:
        out[s.name if s.name == CLASS_KEY else "denoiser." + s.name] = eng.layout.view(src, s.name)
    return out


class JiTTrainLoop:
    """Trainer.training_loop for the JiT class-to-image step. `loader` yields BucketLoader-style batch dicts
    (image fp16 [B,3,h,w] on the device, caption list, original_size / target_size / crop_coords_top_left
    [B,2]); captions are tokenised with the reference's ClassTokenizer (max_token_length)."""

    def __init__(self, trainer: JiTTrainer, optimizer: RAdamScheduleFreeFlat, loader: Iterable, tokenizer: ClassTokenizer,
                 num_train_epochs: int = 1, gradient_accumulation_steps: int = 1, saving: SavingStrategy | None = None,
                 savers: list[SafetensorsSaver] | None = None, use_ema: bool = False, ema_decay: float = 0.9999,
                 sync=None, losslog=None, debug_mode: str | None = None, max_token_length: int | None = None,
                 clip_grad_norm: float | None = None, clip_grad_value: float | None = None):
        self.trainer, self.optimizer, self.loader, self.tokenizer = trainer, optimizer, loader, tokenizer
        self.epochs, self.accum = num_train_epochs, gradient_accumulation_steps
        self.saving, self.savers = saving, list(savers or [])
        self.ema = ParamEMA(trainer.engine.params, ema_decay) if use_ema else None
        # common.py:162-164: the EMA callbacks are copies with the template prefixed by "ema_"
        self.ema_savers = [SafetensorsSaver(s.name, s.save_dir, "ema_" + s.template) for s in self.savers]
        if sync is None:  # single process: the same bucketed step (optimizer overlapped with the backward)
            from .ddp import GradSync, grad_buckets
            world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
            sync = GradSync(trainer.engine.grads, grad_buckets(trainer.engine.layout, trainer.engine.cfg.depth),
                            overlap=world > 1)  # one process: one optimizer launch after the backward is faster
        if clip_grad_norm is not None or clip_grad_value is not None:  # TrainerConfig (src/config.py:74-75)
            sync.configure_clipping(clip_grad_norm, clip_grad_value)
        self.sync, self.losslog, self.debug_mode = sync, losslog, debug_mode
        self._sched = None
        self.max_len = max_token_length or trainer.tcfg.max_token_length
        self.losses: list[float] = []
        self.saved: list[str] = []

    def _step(self, batch, micro: int):
        ids, mask = self.tokenizer.tokenize(batch["caption"], max_length=self.max_len)
        tr = self.trainer
        on_ready = None
        if (micro + 1) % self.accum == 0:  # the synchronising micro-step: reduce + step buckets as they complete
            opt = self.optimizer
            s = self._sched = opt.begin_step()
            self.sync.arm(lambda lo, hi, sc, g, **kw: opt.apply_range(s, lo, hi, sc, g, **kw), 1.0 / self.accum)
            on_ready = self.sync.launch
        loss, _ = tr.step(batch["image"], ids, mask, batch["original_size"], batch["target_size"],
                          batch["crop_coords_top_left"], on_ready=on_ready, accumulate=micro % self.accum != 0)
        return loss

    def _apply_gradients(self):
        """apply_gradients (common.py:380-388): optimizer step with the 1/accum loss scaling (and the DDP mean)
        folded into the update's grad_scale, gradient clipping (after_backward) inside it, EMA update;
        gradients are re-zeroed by the next step's backward."""
        self.sync.launch_rest()
        self.sync.finish()
        self.optimizer.end_step(self._sched)
        if self.ema is not None:
            self.ema.update()

    def _save(self, epoch: int, steps: int):
        """common.py:390-423: wait_for_everyone, save on the main process only, wait_for_everyone (ranks hold
        identical replicas after the synchronised step, so rank 0's copy is the model)."""
        ddp = dist.is_available() and dist.is_initialized()
        if ddp:
            dist.barrier()
        if not ddp or dist.get_rank() == 0:
            meta = {"epoch": str(epoch), "steps": str(steps)}
            sd = reference_state_dict(self.trainer)
            for cb in self.savers:
                self.saved.append(cb.save(sd, epoch, steps, meta))
            if self.ema is not None:
                esd = reference_state_dict(self.trainer, self.ema.ema)
                for cb in self.ema_savers:
                    self.saved.append(cb.save(esd, epoch, steps, meta))
        if ddp:
            dist.barrier()

    def train(self):
        current_step = 0
        for epoch in range(1, self.epochs + 1):
            if hasattr(self.optimizer, "train"):
                self.optimizer.train()  # before_train_epoch (common.py:276-279)
            for micro, batch in enumerate(self.loader):
                current_step += 1
                loss = self._step(batch, current_step - 1)
                if current_step % self.accum == 0:
                    self._apply_gradients()
                if self.losslog is not None:
                    v = self.losslog.push(loss)  # mean over ranks of a step depth-1 pushes ago (or None)
                    if v is not None:
                        self.losses.append(v)
                else:
                    self.losses.append(loss.item())  # the reference's per-step loss.item()
                if self.saving is not None and self.saving.should_save(epoch, current_step):
                    self._save(epoch, current_step)
                if self.debug_mode == "1step":
                    break
            if hasattr(self.optimizer, "eval"):
                self.optimizer.eval()  # after_train_epoch (common.py:281-284)
            if self.debug_mode == "1step":
                break
        if self.losslog is not None:
            while self.losslog.pending:  # the last depth-1 steps' losses
                self.losses.append(self.losslog.pop())
        return current_step
