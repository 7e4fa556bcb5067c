"""The SDXL flow-matching QLoRA training step (BASELINE config 5): SDXLForFlowMatchingTraining.train_step
(train/sdxl/flow_match.py:109-174) with its config defaults (model_prediction / loss_type "velocity",
timestep_sampling scale_shift_sigmoid mean -0.8 std 0.8, noise_scale 1, clean_at_zero False;
flow_match.py:23-31, src/models/sdxl/adapter/flow_match.py:14-19), on latents [B, 4, 128, 128] at 1024^2:

  t   = sample_timestep(...) * 1000                       (flow_match.py:127-140; vpt.timestep, host RNG)
  z, eps = prepare_scaled_noised_latents(x, t / 1000)     (flow_match.py:60-74;   vpt_flow_noise)
  v   = UNet(z, t, context, pooled, sizes)                 (src/models/sdxl/denoiser.py:1007-1240)
  loss = mse(v, eps - x)                                  (flow_match.py:85-96;   vpt_velocity_loss)
  backward -> the 700 LoRA adapters, RAdamScheduleFree   (src/trainer/common.py:308-388)

The UNet's transformer stacks -- the 11 SpatialTransformers, 70 TransformerBlocks, 700 LoRA targets that
SURVEY §8(a) a29/a30 put on the hot path -- are the real thing (vpt.sdxl_train.SDXLStacksQLoRA, NF4 bases,
LoRA r=16). Its conditioning path is the reference's too: sinusoid(t * 1000, 320) -> time_embed MLP,
sinusoid(original_size | crop | target_size, 256) ++ pooled text -> label_emb MLP, summed (denoiser.py:1125-1170),
then per stage SiLU -> Linear(1280 -> C) added per channel, as each ResidualBlock's emb_layers do
(denoiser.py:535-600). The ResNet / conv / resample path between the stacks is NOT on SURVEY §8 (its row 27 OUT)
and is replaced by a frozen skeleton of the same topology: pixel_unshuffle + Linear in place of conv_in and of
each Downsample, Linear + pixel_shuffle for each Upsample and for the out conv, the UNet's skip connections as
additions (the reference concatenates them into its ResNets). Every frozen map runs on the HIP GEMM, forward and
input gradient, so the loss gradient reaches every stack through the whole graph exactly once per step, as in
the reference; the text-encoder states take no gradient (they are computed under no_grad, flow_match.py:115-124).
"""

from __future__ import annotations

import math

import torch

from . import ops
from .sdxl import lora_side_scope
from .sdxl_train import CONTEXT_DIM, CONTEXT_TOKENS, SDXL_1024_STACKS, SDXLStacksQLoRA
from .timestep import sample_timestep

BF16, F32 = torch.bfloat16, torch.float32
POOLED_DIM = 1280
# The reference's SDXL buckets (configs/sdxl/flow_match/config.yml:46-50 -> src/dataset/aspect_ratio_bucket.py:20-60,
# base 1024, step 128, min 384): the five nearest to square, (width, height) in pixels; latents are / 8.
SDXL_BUCKETS_5 = [(1024, 1024), (896, 1152), (1152, 896), (768, 1408), (1408, 768)]


def _check_latent(lat):
    h, w = lat
    if h % 4 or w % 4 or h < 8 or w < 8:
        raise ValueError(f"latent {h}x{w}: both sides must be multiples of 4 (two 2x2 resamplings)")
    if ((h // 4) * (w // 4)) % 8:
        raise ValueError(f"latent {h}x{w}: level-B token count must be a multiple of 8 (transposes, GroupNorm)")
HIDDEN = 320              # UNet hidden_dim: sinusoid width of t, time_embed_dim = 4 x 320
ADDITIONAL_DIM = 256      # additional_cond_dim (the six size conditions)


class _Frozen:
    """A frozen bf16 Linear on the HIP GEMM: forward and input gradient only."""

    def __init__(self, out_f: int, in_f: int, g: torch.Generator, device, bias: bool = True):
        self.w = (torch.randn(out_f, in_f, device=device, generator=g) / math.sqrt(in_f)).to(BF16)
        self.b = (torch.randn(out_f, device=device, generator=g) * 0.02).to(BF16) if bias else None

    def fwd(self, x, out=None, act=ops.ACT_NONE, bias=None, resid=None):
        return ops.linear(x, self.w, bias=self.b if bias is None else bias, resid=resid, out=out, act=act)

    def bwd(self, dy, out=None):
        return ops.linear_dgrad(dy, self.w, out=out)


class SDXLFlowMatchQLoRA:
    """One BASELINE-config-5 training step. `stacks` must follow SDXL's topology: two down stacks at level A
    (latent / 2), two down stacks at level B (latent / 4), the mid stack, three up stacks at B, three up at A
    (SDXL_1024_STACKS: 640 ch at 64 x 64, 1280 ch at 32 x 32 for the square bucket). The step runs ANY
    aspect-ratio bucket: the latent h x w of each step's batch sets the stage shapes (h/2 x w/2, h/4 x w/4); the
    stacks' configured sides only fix the default `latent` (the reference's buckets: configs/sdxl/flow_match/
    config.yml:46-50, bucket_base_size 1024, step 128, min_size 384 -> latents multiples of 16)."""

    def __init__(self, B: int = 4, latent=128, stacks=SDXL_1024_STACKS, n_ctx: int = CONTEXT_TOKENS,
                 context_dim: int = CONTEXT_DIM, rank: int = 16, alpha: float = 1.0, device="cuda", seed: int = 0,
                 lr: float = 1e-3, timestep_sampling: str = "scale_shift_sigmoid", timestep_mean: float = -0.8,
                 timestep_std: float = 0.8, noise_scale: float = 1.0, clean_at_zero: bool = False,
                 emb_dim: int = 4 * HIDDEN, pooled_dim: int = POOLED_DIM, calibrate: bool = True):
        stacks = list(stacks)
        if len(stacks) != 11:
            raise ValueError("SDXL topology: 2 + 2 down, 1 mid, 3 + 3 up stacks")
        cA, sA, cB, sB = stacks[0][1], stacks[0][4], stacks[2][1], stacks[2][4]
        lat = (latent, latent) if isinstance(latent, int) else tuple(latent)
        if sB * 2 != sA or any(s[1] != cA or s[4] != sA for s in stacks[:2] + stacks[8:]) or \
                any(s[1] != cB or s[4] != sB for s in stacks[2:8]):
            raise ValueError("stack channels / sides do not follow the SDXL levels")
        _check_latent(lat)
        self.B, self.latent, self.cA, self.cB = B, lat, cA, cB
        self.n_ctx, self.cdim, self.emb_dim, self.pooled_dim = n_ctx, context_dim, emb_dim, pooled_dim
        self.device = torch.device(device)
        self.core = SDXLStacksQLoRA(B=B, rank=rank, alpha=alpha, stacks=stacks, context_dim=context_dim, n_ctx=n_ctx,
                                    device=device, seed=seed, lr=lr)
        self.sampling = dict(sampling_type=timestep_sampling, mean=timestep_mean, std=timestep_std)
        self.noise_scale, self.clean_at_zero = noise_scale, clean_at_zero
        g = torch.Generator(device=self.device).manual_seed(seed + 7919)
        dev = self.device
        # conditioning MLPs (MLPEmbedder: Linear -> SiLU -> Linear, denoiser.py:20-29), frozen
        self.t1, self.t2 = _Frozen(emb_dim, HIDDEN, g, dev), _Frozen(emb_dim, emb_dim, g, dev)
        self.l1 = _Frozen(emb_dim, pooled_dim + 6 * ADDITIONAL_DIM, g, dev)
        self.l2 = _Frozen(emb_dim, emb_dim, g, dev)
        # per-stage emb_layers (SiLU -> Linear(emb -> channels)) of the three injection points
        self.e_in, self.e_down, self.e_up = (_Frozen(cA, emb_dim, g, dev), _Frozen(cB, emb_dim, g, dev),
                                             _Frozen(4 * cA, emb_dim, g, dev))
        # the skeleton's frozen maps (conv_in, Downsample, Upsample, out conv surrogates)
        self.m_in = _Frozen(cA, 16, g, dev, bias=False)          # pixel_unshuffle(z, 2): 4 x 2 x 2 -> cA
        self.m_down = _Frozen(cB, 4 * cA, g, dev, bias=False)    # pixel_unshuffle(level A, 2) -> cB
        self.m_up = _Frozen(4 * cA, cB, g, dev, bias=False)      # cB -> 4 cA, pixel_shuffle(2) -> level A
        self.m_out = _Frozen(16, cA, g, dev)                     # cA -> 4 x 2 x 2, pixel_shuffle(2) -> latents
        self._seed = seed
        self.gen = torch.Generator().manual_seed(seed + 1)       # timestep sampling (host, like the reference)
        self.step_count = 0
        self.loss = torch.zeros(1, dtype=F32, device=dev)
        self.opt = self.core.opt
        self._probe = None
        if calibrate:
            self.calibrate()

    # ------------------------------------------------------------------ pieces
    def condition(self, t1000: torch.Tensor, pooled: torch.Tensor, sizes: torch.Tensor) -> torch.Tensor:
        """prepare_global_condition (denoiser.py:1125-1170) -> SiLU(global_cond) [B, emb_dim] bf16, the input
        of every emb_layers Linear."""
        B = self.B
        temb = self.t2.fwd(self.t1.fwd(ops.sinusoid_embed(t1000, HIDDEN), act=ops.ACT_SILU))
        add = ops.sinusoid_embed(sizes.reshape(-1).float(), ADDITIONAL_DIM).view(B, 6 * ADDITIONAL_DIM)
        gin = torch.cat([pooled.to(BF16), add], 1)  # [B, pooled_dim + 1536] (torch.cat order of the reference)
        glob = self.l2.fwd(self.l1.fwd(gin, act=ops.ACT_SILU), resid=temb)  # label_emb(...) + time_embed
        return ops.silu(glob, torch.empty_like(glob))

    def _map_per_sample(self, lin: _Frozen, x_tok: torch.Tensor, emb: torch.Tensor, n_tok: int) -> torch.Tensor:
        """y[b] = lin(x_tok[b]) + emb[b] (the per-sample, per-channel embedding add, in the GEMM's bias)."""
        out = torch.empty(self.B * n_tok, lin.w.shape[0], dtype=BF16, device=self.device)
        for b in range(self.B):
            lin.fwd(x_tok[b * n_tok:(b + 1) * n_tok], out=out[b * n_tok:(b + 1) * n_tok], bias=emb[b])
        return out

    def _capture(self, name: str, x: torch.Tensor):
        if self._probe is not None and name not in self._probe:
            self._probe[name] = float(x.float().pow(2).mean().sqrt())

    @torch.no_grad()
    def calibrate(self, seed: int = 4242):
        """Unit-RMS outputs for the skeleton maps that read un-normalised residual sums (Downsample, Upsample and
        out-conv surrogates: m_down, m_up, m_out), one forward each on a calibration batch, in graph order. The
        UNet's ResNets renormalise (GroupNorm) what its skips concatenate; the skeleton's additions do not, and
        without this the residual stream grows through the 70 blocks and 5 skips until the velocity MSE sits in
        the hundreds on unit-variance targets. Everything the stacks' GEMMs read stays normalised (GroupNorm /
        LayerNorm outputs) either way; this only sets the magnitudes of the residual stream and of v."""
        lat, ctx, pooled, sizes = self.make_inputs(seed=seed)
        t = torch.full((self.B,), 0.5, device=self.device)
        for name in ("m_down", "m_up", "m_out"):
            self._probe = {}
            self.step(lat, ctx, pooled, sizes, t=t, backward=False)
            rms = self._probe[name]
            lin = getattr(self, name)
            k = 1.0 / max(rms, 1e-6)  # the map's N(0, 1/in) weights keep the RMS of their input
            lin.w = (lin.w.float() * k).to(BF16)
        self._probe = None
        self.step_count = 0
        self.gen = torch.Generator().manual_seed(self._seed + 1)

    def _levels(self, Lh: int, Lw: int):
        """Stage sides of a latent h x w: level A (h/2 x w/2) and level B (h/4 x w/4)."""
        _check_latent((Lh, Lw))
        return (Lh // 2, Lw // 2), (Lh // 4, Lw // 4)

    def forward(self, z: torch.Tensor, ctx: torch.Tensor, sg: torch.Tensor) -> torch.Tensor:
        """The UNet on z [B, 4, h, w] bf16 -> v [B, 4, h, w] bf16 (activations kept for backward)."""
        B, cA, cB = self.B, self.cA, self.cB
        Lh, Lw = z.shape[2], z.shape[3]
        (ah, aw), (bh, bw) = self._levels(Lh, Lw)
        hA, hB = ah * aw, bh * bw
        S = [st for (_, _, _, st) in self.core.stacks]
        nc = self.n_ctx
        self.core.precompute_ctx_kv(ctx)  # every block's cross-attention k / v of the fixed context, stacked GEMMs
        eA, eB, eU = self.e_in.fwd(sg), self.e_down.fwd(sg), self.e_up.fwd(sg)
        tok = ops.space_to_depth(z, B, 4, Lh, Lw, 2).view(B * hA, 16)
        x64 = ops.transpose_add(self._map_per_sample(self.m_in, tok, eA, hA).view(B, hA, cA), B, hA, cA)
        e0 = S[0].forward(x64, ctx, B, hA, nc)
        e1 = S[1].forward(e0, ctx, B, hA, nc)
        tok = ops.space_to_depth(e1, B, cA, ah, aw, 2).view(B * hB, 4 * cA)
        self._capture("m_down", tok)
        x32 = ops.transpose_add(self._map_per_sample(self.m_down, tok, eB, hB).view(B, hB, cB), B, hB, cB)
        d0 = S[2].forward(x32, ctx, B, hB, nc)
        d1 = S[3].forward(d0, ctx, B, hB, nc)
        m = S[4].forward(d1, ctx, B, hB, nc)
        u0 = S[5].forward(ops.add_bf16(m, d1), ctx, B, hB, nc)
        u1 = S[6].forward(ops.add_bf16(u0, d0), ctx, B, hB, nc)
        u2 = S[7].forward(ops.add_bf16(u1, x32), ctx, B, hB, nc)
        tok = ops.transpose_add(u2, B, cB, hB).view(B * hB, cB)
        self._capture("m_up", tok)
        y64 = ops.space_to_depth(self._map_per_sample(self.m_up, tok, eU, hB), B, cA, ah, aw, 2, inverse=True)
        y64 = y64.view(B, cA, hA)
        v0 = S[8].forward(ops.add_bf16(y64, e1), ctx, B, hA, nc)
        v1 = S[9].forward(ops.add_bf16(v0, e0), ctx, B, hA, nc)
        v2 = S[10].forward(ops.add_bf16(v1, x64), ctx, B, hA, nc)
        tok = ops.transpose_add(v2, B, cA, hA).view(B * hA, cA)
        self._capture("m_out", tok)
        return ops.space_to_depth(self.m_out.fwd(tok), B, 4, Lh, Lw, 2, inverse=True)

    def backward(self, dv: torch.Tensor):
        """dL/dv [B, 4, h, w] -> every adapter gradient (the skeleton is frozen; no input gradient needed)."""
        B, cA, cB = self.B, self.cA, self.cB
        Lh, Lw = dv.shape[2], dv.shape[3]
        (ah, aw), (bh, bw) = self._levels(Lh, Lw)
        hA, hB = ah * aw, bh * bw
        S = [st for (_, _, _, st) in self.core.stacks]
        add = ops.add_bf16

        def back(i, dy):
            return S[i].backward(dy, need_dctx=False)[0]

        d = self.m_out.bwd(ops.space_to_depth(dv, B, 4, Lh, Lw, 2).view(B * hA, 16))
        dv2 = ops.transpose_add(d.view(B, hA, cA), B, hA, cA)
        dsum = back(10, dv2)                      # d(v1 + x64)
        dx64 = dsum
        dsum = back(9, dsum)                      # d(v0 + e0)
        de0 = dsum
        dsum = back(8, dsum)                      # d(y64 + e1)
        de1 = dsum
        tok = ops.space_to_depth(dsum.view(B, cA, ah, aw), B, cA, ah, aw, 2).view(B * hB, 4 * cA)
        du2 = ops.transpose_add(self.m_up.bwd(tok).view(B, hB, cB), B, hB, cB)
        dsum = back(7, du2)                       # d(u1 + x32)
        dx32 = dsum
        dsum = back(6, dsum)                      # d(u0 + d0)
        dd0 = dsum
        dsum = back(5, dsum)                      # d(m + d1)
        dd1 = add(back(4, dsum), dsum)            # mid, plus the skip
        dd0 = add(back(3, dd1), dd0)
        dx32 = add(back(2, dd0), dx32)
        tok = ops.transpose_add(dx32, B, cB, hB).view(B * hB, cB)
        de1 = add(ops.space_to_depth(self.m_down.bwd(tok), B, cA, ah, aw, 2, inverse=True).view(B, cA, hA), de1)
        de0 = add(back(1, de1), de0)
        back(0, de0)                               # (+ dx64: the input map is frozen, z needs no gradient)

    # ------------------------------------------------------------------ the step
    def sample_t(self, shape=None) -> torch.Tensor:
        """sample_timestep(latents.shape, ...) (flow_match.py:127-140), t in (0, 1) f32 [B] on the device. `shape` = the
        batch's latent shape (resolution-dependent samplers such as flux_shift use its h, w); default the model's."""
        shape = tuple(shape) if shape is not None else (self.B, 4, *self.latent)
        return sample_timestep(shape, "cpu", generator=self.gen, **self.sampling).to(self.device)

    def step(self, latents: torch.Tensor, ctx: torch.Tensor, pooled: torch.Tensor, sizes: torch.Tensor,
             t: torch.Tensor | None = None, eps: torch.Tensor | None = None, backward: bool = True,
             optimizer_step: bool = True):
        """latents bf16 [B, 4, L, L]; ctx bf16 [B * n_ctx, context_dim]; pooled [B, 1280]; sizes [B, 6]
        (original_size, crop_coords_top_left, target_size). Returns (loss device f32 [1], v)."""
        B = self.B
        t = self.sample_t(latents.shape) if t is None else t.to(self.device, F32)
        t1000 = t * 1000.0                          # the model's timestep (0~1000)
        z = torch.empty_like(latents)
        eps_buf = torch.empty_like(latents) if eps is None else None
        seed = (self.step_count * 1000003 + 12345) & 0x7FFFFFFFFFFF
        self.step_count += 1
        ops.flow_noise(latents, t, B, z, eps=eps_buf, eps_in=eps, noise_scale=self.noise_scale,
                       clean_at_zero=self.clean_at_zero, seed=seed)
        eps = eps if eps is not None else eps_buf
        sg = self.condition(t1000, pooled, sizes)
        if backward:
            self.core.grads.zero_()
        v = self.forward(z, ctx, sg)
        dv = torch.empty_like(v) if backward else None
        ops.velocity_loss(v, latents, eps, self.loss, dv)
        if backward:
            with lora_side_scope(self.device):  # adapter gradients beside the chain, joined before anything reads them
                self.backward(dv)
            if optimizer_step:
                self.opt.step()
        self._last = dict(t=t, z=z, eps=eps)
        return self.loss, v

    def make_inputs(self, seed: int = 1, latent=None):
        """Synthetic batch of one bucket: VAE latents (scaled, ~unit variance) bf16 [B, 4, h, w] (latent = (h, w),
        default the model's), the 231 x 2048 text context, the pooled CLIP-G output, and the size conditions
        (original_size = target_size = (8h, 8w), crop (0, 0); text_to_image.py:198-217 order (height, width))."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        B = self.B
        Lh, Lw = self.latent if latent is None else ((latent, latent) if isinstance(latent, int) else latent)
        _check_latent((Lh, Lw))
        lat = torch.randn(B, 4, Lh, Lw, device=self.device, generator=g).to(BF16)
        ctx = torch.randn(B * self.n_ctx, self.cdim, device=self.device, generator=g).to(BF16)
        pooled = torch.randn(B, self.pooled_dim, device=self.device, generator=g).to(BF16)
        sizes = torch.tensor([[8 * Lh, 8 * Lw, 0, 0, 8 * Lh, 8 * Lw]] * B, dtype=F32, device=self.device)
        return lat, ctx, pooled, sizes

    def flops_per_step(self, latent=None) -> float:
        """Algorithmic FLOPs of one step at a latent h x w (default the model's): the stacks' (vpt.sdxl_train) plus
        the skeleton's GEMMs, forward + input grad."""
        Lh, Lw = self.latent if latent is None else latent
        (ah, aw), (bh, bw) = self._levels(Lh, Lw)
        B, hA, hB, cA, cB = self.B, ah * aw, bh * bw, self.cA, self.cB
        f = self.core.flops_per_step(hws=[hA if s[1] == cA and i in (0, 1, 8, 9, 10) else hB
                                          for i, s in enumerate(self.core.stacks)])
        f += 2 * (2 * B * hA * 16 * cA) * 2 + 2 * (2 * B * hB * 4 * cA * cB) * 2  # in / out, down / up maps
        return f

    def n_adapter_params(self) -> int:
        return self.core.n_adapter_params()
