"""HipDenoiser: drop-in replacement for the reference JiT denoiser class.

Swap point: `JiTModel.denoiser_class` (src/models/jit/pipeline.py:19-21). HipDenoiser has
  * the constructor `(config: DenoiserConfig)` (reference pydantic config objects are accepted),
  * `forward(image, timestep, context, original_size, target_size, crop_coords, context_mask=None)
    -> [B, C, H, W]` (src/models/jit/denoiser.py:969-978),
  * `initialize_weights()` (764-798) and `set_gradient_checkpointing()` (800-801),
  * the reference state-dict names and shapes (parameters are views into one flat bf16 buffer).
Forward and backward each run as one HIP schedule (vpt.engine.JiTEngine) wrapped in a single
autograd.Function, so `loss.backward()` from the unchanged reference training step fills `.grad`
of every parameter and of `context` (the class-embedding output).
"""

from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from .config import DenoiserConfig
from .engine import JiTEngine

BF16, F32 = torch.bfloat16, torch.float32


def _as_config(config) -> DenoiserConfig:
    if isinstance(config, DenoiserConfig):
        return config
    if hasattr(config, "model_dump"):
        return DenoiserConfig.model_validate(config.model_dump())
    return DenoiserConfig.model_validate(dict(config))


class _JiTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod: "HipDenoiser", image, timestep, context, original_size, target_size, crop_coords,
                context_mask, *params):
        eng = mod.engine
        B, C, H, W = image.shape
        save = torch.is_grad_enabled() or any(p.requires_grad for p in params) or context.requires_grad
        out = mod._forward_engine(image, timestep, context, original_size, target_size, crop_coords, context_mask,
                                  save=save)
        img = torch.empty(B, C, H, W, dtype=BF16, device=image.device)
        ops.unpatchify(out, B, H, W, img)
        ctx.mod = mod
        ctx.gen = mod._gen
        ctx.shape = (B, C, H, W)
        ctx.ctx_shape = context.shape
        ctx.ctx_dtype = context.dtype
        return img

    @staticmethod
    def backward(ctx, grad_img):
        mod: HipDenoiser = ctx.mod
        if ctx.gen != mod._gen:
            raise RuntimeError("HipDenoiser keeps the activations of its most recent forward only: call backward() "
                               "before running another forward with autograd enabled")
        eng = mod.engine
        B, C, H, W = ctx.shape
        np_ = (H // 16) * (W // 16)
        dout = eng.pool.get("api_dout", (B * np_, C * 256))
        ops.unpatchify(dout, B, H, W, grad_img.to(BF16).contiguous(), reverse=True)
        dctx = eng.backward(dout)
        grads = [eng.g[n].to(p.dtype) if p.requires_grad else None for n, p in mod._named]
        dcontext = None
        if dctx is not None and ctx.needs_input_grad[3]:
            dcontext = dctx.view(ctx.ctx_shape).to(ctx.ctx_dtype)
        return (None, None, None, dcontext, None, None, None, None, *grads)


class HipDenoiser(nn.Module):
    def __init__(self, config, device: str | torch.device = "cuda"):
        super().__init__()
        self.config = _as_config(config)
        self.engine = JiTEngine(self.config, device=device, n_classes=None)
        self.gradient_checkpointing = False
        self._gen = 0
        self._named: list[tuple[str, nn.Parameter]] = []
        self._build_params()

    # parameters are registered under the reference's module paths, as views of the flat buffer
    def _build_params(self):
        self._named = []
        for s in self.engine.layout.specs:
            *path, leaf = s.name.split(".")
            mod = self
            for part in path:
                if part not in mod._modules:
                    mod.add_module(part, nn.Module())
                mod = mod._modules[part]
            p = nn.Parameter(self.engine.p[s.name], requires_grad=True)
            mod.register_parameter(leaf, p)
            self._named.append((s.name, p))

    def _apply(self, fn, recurse=True):
        # .to()/.cuda()/.bfloat16() must not break the aliasing with the engine's flat buffer: apply
        # fn to a copy of every parameter, write it back into the flat buffer, keep the views.
        for name, p in self._named:
            new = fn(p.data)
            if new.device != self.engine.device:
                raise ValueError("HipDenoiser lives on its construction device; build it on the target GPU")
            self.engine.p[name].copy_(new.to(BF16))
        return self

    def initialize_weights(self, seed: int = 0):
        self.engine.init_weights(seed)

    def set_gradient_checkpointing(self, enable: bool = True):
        """denoiser.py:800-801 + forward_block 945-967: keep only the block inputs in training forwards and
        recompute each block's intermediates in backward (identical gradients: the kernels are deterministic)."""
        self.gradient_checkpointing = enable
        self.engine.set_gradient_checkpointing(enable)

    def _forward_engine(self, image, timestep, context, original_size, target_size, crop_coords, context_mask,
                        save: bool):
        eng, cfg = self.engine, self.config
        B, C, H, W = image.shape
        dev = eng.device
        hp, wp, np_, rows = eng.shape_info(B, H, W, context.shape[1])
        n_ctx = context.shape[1]
        pool = eng.pool if save else eng.pool_infer
        zp = pool.get("api_zp", (B * np_, C * 256))
        ops.patchify(image.to(device=dev, dtype=BF16).contiguous(), B, H, W, zp, noising=False)
        t_vals = (timestep.to(dev) * cfg.timestep_scale).float().contiguous()
        size_vals = torch.cat([original_size, target_size, crop_coords], 1).reshape(-1).to(dev, F32).contiguous()
        ctx_raw = context.to(device=dev, dtype=BF16).reshape(B * n_ctx, -1).contiguous()
        kbias = None
        if context_mask is not None:
            n_pre = np_ + 6 + cfg.num_time_tokens
            kbias = pool.get("api_kbias", (B, rows), F32)
            kbias[:, :n_pre].zero_()
            kbias[:, n_pre:] = torch.where(context_mask.to(dev).bool(), 0.0, float("-inf"))
        if save:
            self._gen += 1
        return eng.forward(zp, B, H, W, t_vals, size_vals, ctx_raw, kbias, n_ctx, save=save)

    def forward(self, image, timestep, context, original_size, target_size, crop_coords, context_mask=None):
        params = [p for _, p in self._named]
        return _JiTFunction.apply(self, image, timestep, context, original_size, target_size, crop_coords,
                                  context_mask, *params)


# reference name of the swap-in class (src/models/jit/denoiser.py:1127-1130)
Denoiser = HipDenoiser
