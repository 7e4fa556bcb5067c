"""Euler + classifier-free-guidance sampler on the HIP engine -- JiTModel.generate
(src/models/jit/pipeline.py:378-488) for class-conditioned JiT.

Per denoising step: one inference forward of the engine (no saved activations, its own buffer
pool) over [z; z] (CFG) or z, then one fused kernel (`vpt_euler_cfg_step`) that reads the
prediction in patch layout and updates the bf16 image in place with the reference's bf16 rounding.
Everything on the device; the only host work is tokenisation and the step schedule.
"""

from __future__ import annotations

import torch

from . import ops
from .engine import JiTEngine
from .jit_train import ClassTokenizer

BF16 = torch.bfloat16
F32 = torch.float32


class JiTSampler:
    """`engine` holds the denoiser + class-embedding weights (reference state-dict names);
    `tokenizer` mirrors ClassTokenizer (src/models/jit/class_encoder.py:42-90);
    `model_pred` mirrors JiTConfig.model_pred ("image" or "velocity")."""

    def __init__(self, engine: JiTEngine, tokenizer: ClassTokenizer, model_pred: str = "image"):
        if model_pred not in ("image", "velocity"):
            raise NotImplementedError(f"model_pred={model_pred!r} (reference: noise prediction is not implemented)")
        if "class_encoder.embedding.weight" not in engine.p:
            raise ValueError("the engine was built without a class embedding (n_classes)")
        self.engine = engine
        self.tokenizer = tokenizer
        self.model_pred = model_pred
        self.device = engine.device

    @staticmethod
    def _prompts(p):
        return p if isinstance(p, list) else [p]

    @torch.inference_mode()
    def generate(self, prompt, negative_prompt=None, width: int = 256, height: int = 256,
                 num_inference_steps: int = 20, cfg_scale: float = 2.0, max_token_length: int = 64,
                 seed: int | None = None, noise: torch.Tensor | None = None, do_cfg_renorm: bool = False,
                 do_dynamic_thresholding: bool = False, cfg_time_range=(0.0, 1.0)) -> torch.Tensor:
        """Returns the final image [B, 3, height, width] bf16 on the device (the reference converts it
        to PIL at this point, pipeline.py:483-486). `noise` overrides the seeded starting image."""
        if do_cfg_renorm or do_dynamic_thresholding:
            raise NotImplementedError("cfg renorm / dynamic thresholding are not on the HIP sampler path")
        eng, cfg = self.engine, self.engine.cfg
        prompts = self._prompts(prompt)
        B = len(prompts)
        H, W = height, width
        do_cfg = cfg_scale > 1.0
        timesteps = torch.linspace(0.0, 1.0, num_inference_steps + 1)          # pipeline.py:150-161
        if noise is None:                                                       # pipeline.py:124-148
            gen = None
            if seed is not None:
                gen = torch.Generator(device=self.device).manual_seed(seed)
            z = torch.randn((B, 3, H, W), dtype=BF16, device=self.device, generator=gen)
        else:
            z = noise.to(device=self.device, dtype=BF16).clone()
        neg = self._prompts(negative_prompt) if negative_prompt is not None else [""]
        if len(neg) == 1 and B != 1:
            neg = neg * B
        pos_ids, pos_mask = self.tokenizer.tokenize(prompts, max_length=max_token_length)
        neg_ids, _ = self.tokenizer.tokenize(neg, max_length=max_token_length)
        # negative embeddings are paired with the POSITIVE mask (pipeline.py:193-219)
        ids = torch.cat([pos_ids, neg_ids]) if do_cfg else pos_ids
        mask = torch.cat([pos_mask, pos_mask]) if do_cfg else pos_mask
        n_all, n_ctx = ids.shape
        pool = eng.pool_infer
        ctx_all = ops.embed_gather(eng.p["class_encoder.embedding.weight"], ids.to(self.device),
                                   pool.get("s_ctx", (n_all * n_ctx, cfg.context_dim)))
        hp, wp, np_, rows = eng.shape_info(n_all, H, W, n_ctx)
        n_pre = np_ + 6 + cfg.num_time_tokens
        kb_all = torch.zeros(n_all, rows, dtype=F32, device=self.device)
        kb_all[:, n_pre:n_pre + n_ctx] = torch.where(mask.to(self.device).bool(), 0.0, float("-inf"))
        size_all = torch.tensor([H, W, H, W, 0, 0], dtype=F32, device=self.device).repeat(n_all)
        zp = pool.get("s_zp", (n_all * np_, 3 * cfg.patch_size ** 2))
        mode = 0 if self.model_pred == "image" else 1
        for i in range(num_inference_steps):
            t = float(timesteps[i])
            in_cfg = do_cfg and cfg_time_range[0] <= t <= cfg_time_range[1]   # pipeline.py:437-439
            n = 2 * B if in_cfg else B
            ops.patchify(z, B, H, W, zp[: B * np_], noising=False)
            if in_cfg:
                zp[B * np_: 2 * B * np_].copy_(zp[: B * np_])
            t_vals = torch.full((n,), t * cfg.timestep_scale, dtype=F32, device=self.device)
            out = eng.forward(zp[: n * np_], n, H, W, t_vals, size_all[: 6 * n], ctx_all[: n * n_ctx],
                              kb_all[:n], n_ctx, save=False)
            dt = float(timesteps[i + 1] - timesteps[i])
            ops.euler_cfg_step(z, out, B, H, W, in_cfg, cfg_scale, mode, t, dt)
        return z

    @staticmethod
    def to_uint8(images: torch.Tensor) -> torch.Tensor:
        """[-1, 1] images -> uint8 [B, H, W, 3], as the reference's tensor_to_images
        (src/utils/tensor.py:91-105): arithmetic in the image dtype, then truncation to uint8."""
        x = (images.clamp(-1.0, 1.0) + 1.0) / 2.0 * 255.0
        return x.permute(0, 2, 3, 1).float().to(torch.uint8).contiguous()
