"""CPU ORACLE (test infrastructure only — never imported by the product path).

A from-scratch fp32 PyTorch-CPU restatement of the reference JiT rectified-flow training step,
used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker. Each
function cites the reference file:line (paths relative to p1atdev/vision-pt) it restates.

Parity pinned: against golden vectors generated from the reference itself in the survey
container (tests/golden/make_golden.py, fixtures in tests/golden/*.safetensors) and the
reference's own known-answer tests (tests/models/test_jit.py:32-71 timestep embedding,
tests/test_dataset.py:19-44 bucket counts, tests/test_patch.py:17-89 patchify round trip).

Numerics mirror the reference in fp32 mode: f32 everywhere except the q/k/v cast to bf16
before SDPA (src/modules/attention.py:113-118).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F


# ------------------------------------------------------------------------------- config
@dataclass
class OracleConfig:
    """Subset of DenoiserConfig (src/models/jit/config.py:16-46) that the JiT-B path uses."""
    patch_size: int = 16
    in_channels: int = 3
    out_channels: int = 3
    hidden_size: int = 768
    depth: int = 12
    num_heads: int = 12
    mlp_ratio: float = 4.0
    bottleneck_dim: int = 128
    num_time_tokens: int = 4
    timestep_scale: float = 1.0
    rope_theta: float = 256.0
    rope_axes_dims: list = field(default_factory=lambda: [16, 24, 24])
    rope_axes_lens: list = field(default_factory=lambda: [256, 128, 128])
    rope_zero_centered: list = field(default_factory=lambda: [False, True, True])
    context_dim: int = 768
    context_start_block: int = 4
    do_context_fuse: bool = False

    @property
    def mlp_hidden(self) -> int:
        # SwiGLU hidden = int(int(D * mlp_ratio) * 2 / 3)   (denoiser.py:490, 641-646)
        return int(int(self.hidden_size * self.mlp_ratio) * 2 / 3)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads


def jit_b16() -> OracleConfig:
    """JiT_B_16_Config (src/models/jit/config.py:49-65)."""
    return OracleConfig()


# ------------------------------------------------------------------------------- embeddings
def timestep_embedding(t: torch.Tensor, dim: int = 256, max_period: int = 10000) -> torch.Tensor:
    """get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0)
    (src/modules/timestep/embedding.py:10-62)."""
    half = dim // 2
    expo = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32)
    expo = expo / half
    emb = t[:, None].float() * torch.exp(expo)[None, :]
    return torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)


def rope_axis_table(dim: int, lo: int, hi: int, theta: float) -> torch.Tensor:
    """RopeEmbedder.get_rope_freqs (denoiser.py:141-177): angles in f64, cast f32, polar -> c64."""
    freqs = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    pos = torch.arange(lo, hi, dtype=torch.float64)
    ang = torch.outer(pos, freqs).float()
    return torch.polar(torch.ones_like(ang), ang).to(torch.complex64)


def rope_freqs(cfg: OracleConfig, h_p: int, w_p: int, n_ctx: int) -> torch.Tensor:
    """freqs_cis [N, head_dim/2] complex64 in token order patches | size(6) | time(T) | context
    (denoiser.py:1013-1051; ids: prepare_image_position_ids 228-268, context ids 270-287)."""
    tables, offs = [], []
    for dim, ln, zc in zip(cfg.rope_axes_dims, cfg.rope_axes_lens, cfg.rope_zero_centered):
        lo, hi = ((ln // 2) - ln, ln // 2) if zc else (0, ln)
        tables.append(rope_axis_table(dim, lo, hi, cfg.rope_theta))
        offs.append(ln // 2 if zc else 0)

    def lookup(ids: torch.Tensor) -> torch.Tensor:
        parts = []
        for a in range(3):
            idx = ids[:, a].long() + offs[a]
            if (idx < 0).any() or (idx >= tables[a].shape[0]).any():
                raise IndexError(f"rope axis {a}: position out of range (bucket too large)")
            parts.append(tables[a][idx])
        return torch.cat(parts, dim=-1)

    ys = torch.arange(h_p // 2 - h_p, h_p // 2).view(-1, 1).expand(h_p, w_p)
    xs = torch.arange(w_p // 2 - w_p, w_p // 2).view(1, -1).expand(h_p, w_p)
    img = torch.stack([torch.full_like(ys, 3), ys, xs], -1).reshape(-1, 3)

    def seq(n: int, gidx: int) -> torch.Tensor:
        a = torch.arange(n)
        return torch.stack([torch.full_like(a, gidx), a, a], -1)

    return torch.cat([lookup(img), lookup(seq(6, 2)), lookup(seq(cfg.num_time_tokens, 1)), lookup(seq(n_ctx, 0))], 0)


def apply_rope(x: torch.Tensor, freqs: torch.Tensor) -> torch.Tensor:
    """denoiser.py:98-111 — x [B,H,N,hd] (pairs interleaved), freqs [N,hd/2] c64."""
    B, H, N, D = x.shape
    xc = torch.view_as_complex(x.float().reshape(B, H, N, D // 2, 2))
    return torch.view_as_real(xc * freqs[None, None]).flatten(3).type_as(x)


# ------------------------------------------------------------------------------- modules
class RMSNorm(nn.Module):
    """FP32RMSNorm (src/modules/norm.py:20-27)."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x):
        return F.rms_norm(x.float(), (x.shape[-1],), weight=self.weight, eps=self.eps).to(x.dtype)


class PatchEmbed(nn.Module):
    """BottleneckPatchEmbed (denoiser.py:17-67)."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        p = cfg.patch_size
        self.proj_1 = nn.Conv2d(cfg.in_channels, cfg.bottleneck_dim, p, p, bias=False)
        self.proj_2 = nn.Conv2d(cfg.bottleneck_dim, cfg.hidden_size, 1, 1, bias=True)

    def forward(self, x):
        return self.proj_2(self.proj_1(x)).flatten(2).transpose(1, 2)


class TimeMLP(nn.Module):
    """TimestepEmbedder (denoiser.py:70-95)."""

    def __init__(self, hidden: int):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(256, hidden), nn.SiLU(), nn.Linear(hidden, hidden))

    def forward(self, t):
        return self.mlp(timestep_embedding(t).to(self.mlp[0].weight.dtype))


class SwiGLU(nn.Module):
    """denoiser.py:480-506."""

    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.w_1 = nn.Linear(dim, hidden)
        self.w_2 = nn.Linear(dim, hidden)
        self.w_3 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.w_3(F.silu(self.w_1(x)) * self.w_2(x))


class Attention(nn.Module):
    """denoiser.py:290-397 with scaled_dot_product_attention (src/modules/attention.py:98-129)."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        D = cfg.hidden_size
        self.h = cfg.num_heads
        self.q_norm = RMSNorm(cfg.head_dim)
        self.k_norm = RMSNorm(cfg.head_dim)
        self.to_q, self.to_k, self.to_v, self.to_o = (nn.Linear(D, D) for _ in range(4))

    def forward(self, x, freqs, mask):
        B, N, D = x.shape

        def heads(t):
            return t.view(B, N, self.h, D // self.h).permute(0, 2, 1, 3)

        q, k, v = heads(self.to_q(x)), heads(self.to_k(x)), heads(self.to_v(x))
        q = apply_rope(self.q_norm(q), freqs)
        k = apply_rope(self.k_norm(k), freqs)
        if q.dtype == torch.float32:  # attention.py:113-118: SDPA always runs in bf16
            q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
        m = mask.bool().view(B, 1, 1, N).expand(-1, self.h, N, -1)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=m).to(x.dtype)
        return self.to_o(o.permute(0, 2, 1, 3).reshape(B, N, D))


class Block(nn.Module):
    """JiTBlock (denoiser.py:582-649)."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.norm1 = RMSNorm(cfg.hidden_size)
        self.attn = Attention(cfg)
        self.norm2 = RMSNorm(cfg.hidden_size)
        self.mlp = SwiGLU(cfg.hidden_size, cfg.mlp_hidden)

    def forward(self, x, freqs, mask):
        x = x + self.attn(self.norm1(x), freqs, mask)
        return x + self.mlp(self.norm2(x))


class FinalLayer(nn.Module):
    """denoiser.py:509-543."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.norm_final = RMSNorm(cfg.hidden_size)
        self.mlp = SwiGLU(cfg.hidden_size, cfg.mlp_hidden)
        self.linear = nn.Linear(cfg.hidden_size, cfg.patch_size ** 2 * cfg.out_channels)

    def forward(self, x):
        return self.linear(self.mlp(self.norm_final(x)))


class OracleJiT(nn.Module):
    """JiT (denoiser.py:652-1124) — identical parameter names, so state_dicts are interchangeable
    with the reference `Denoiser` and with vpt's HIP denoiser."""

    def __init__(self, cfg: OracleConfig):
        super().__init__()
        self.config = cfg
        D = cfg.hidden_size
        self.patch_embedder = PatchEmbed(cfg)
        self.time_embedder = TimeMLP(D)
        self.time_position_embeds = nn.Parameter(torch.zeros(cfg.num_time_tokens, D))
        self.image_size_embedder = TimeMLP(D)
        self.context_embedder = nn.Linear(cfg.context_dim, D)
        self.blocks = nn.ModuleList(Block(cfg) for _ in range(cfg.depth))
        self.final_layer = FinalLayer(cfg)

    def forward(self, image, timestep, context, original_size, target_size, crop_coords, context_mask=None):
        cfg = self.config
        B, _, H, W = image.shape
        p = cfg.patch_size
        # time tokens (denoiser.py:982-993)
        te = self.time_embedder(timestep * cfg.timestep_scale)
        time_tokens = te.unsqueeze(1) + self.time_position_embeds.unsqueeze(0)
        ctx = self.context_embedder(context)                                 # 997
        size_info = torch.cat([original_size, target_size, crop_coords], 1).view(-1)
        size_tok = self.image_size_embedder(size_info).view(B, 6, -1)       # 914-943
        patches = self.patch_embedder(image)                                 # 1009
        n_p, n_ctx = patches.shape[1], ctx.shape[1]
        freqs = rope_freqs(cfg, H // p, W // p, n_ctx)
        if context_mask is None:                                             # 1054-1075
            cm = torch.ones(B, n_ctx)
        else:
            cm = context_mask.float()
        mask = torch.cat([torch.ones(B, n_p + 6 + cfg.num_time_tokens), cm], 1)
        tokens = torch.cat([patches, size_tok, time_tokens], 1)              # 1078-1085
        for i, blk in enumerate(self.blocks):                                # 1087-1113
            add = i == cfg.context_start_block or (not cfg.do_context_fuse and i >= cfg.context_start_block)
            if add:
                tokens = torch.cat([tokens, ctx], 1)
            n = tokens.shape[1]
            tokens = blk(tokens, freqs[:n], mask[:, :n])
            if not cfg.do_context_fuse and i >= cfg.context_start_block:
                tokens = tokens[:, :-n_ctx]
        out = self.final_layer(tokens[:, :n_p])
        return unpatchify(out, H, W, p, cfg.out_channels)


def unpatchify(x: torch.Tensor, H: int, W: int, p: int = 16, c: int = 3) -> torch.Tensor:
    """JiT._unpatchify (denoiser.py:828-860): per-patch (py, px, c) -> NCHW."""
    B = x.shape[0]
    return x.view(B, H // p, W // p, p, p, c).permute(0, 5, 1, 3, 2, 4).reshape(B, c, H, W)


def patchify_conv_order(img: torch.Tensor, p: int = 16) -> torch.Tensor:
    """Conv2d(k=p, s=p) im2col layout (c, ky, kx) per patch, row-major patches."""
    B, C, H, W = img.shape
    return img.view(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5).reshape(B, (H // p) * (W // p), C * p * p)


# ------------------------------------------------------------------------------- init / weights
def make_weights(cfg: OracleConfig, seed: int, n_classes: int | None = None) -> dict[str, torch.Tensor]:
    """Deterministic synthetic weights by parameter name (test vectors only): N(0, 0.02) for
    matrices/embeddings as initialize_weights (denoiser.py:764-798) draws them, but biases and
    norm weights are randomised too so every parameter is exercised."""
    g = torch.Generator().manual_seed(seed)
    model = OracleJiT(cfg)
    out = {}
    for name, prm in model.state_dict().items():
        if name.endswith("norm.weight") or name.endswith("norm1.weight") or name.endswith("norm2.weight") \
                or name.endswith("norm_final.weight") or name.endswith("q_norm.weight") or name.endswith("k_norm.weight"):
            out[name] = 1.0 + 0.1 * torch.randn(prm.shape, generator=g)
        elif name.endswith("bias"):
            out[name] = 0.02 * torch.randn(prm.shape, generator=g)
        else:
            out[name] = 0.02 * torch.randn(prm.shape, generator=g)
    if n_classes is not None:
        out["class_encoder.embedding.weight"] = 0.02 * torch.randn(n_classes + 1, cfg.context_dim, generator=g)
    return out


def load_weights(model: nn.Module, weights: dict[str, torch.Tensor]) -> nn.Module:
    sd = {k: v for k, v in weights.items() if not k.startswith("class_encoder.")}
    model.load_state_dict(sd, strict=True)
    return model


# ------------------------------------------------------------------------------- flow matching step
def scale_shift_sigmoid(n: torch.Tensor, mean: float = -0.8, std: float = 0.8) -> torch.Tensor:
    """src/modules/timestep/sampling.py:259-272 with the randn draw passed in."""
    return (n * std + mean).sigmoid()


def noised(x: torch.Tensor, t: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
    """prepare_scaled_noised_latents (src/modules/loss/flow_match.py:60-74), clean_at_zero=False."""
    tt = t.view(-1, *([1] * (x.dim() - 1)))
    return tt * x + (1 - tt) * noise


def image_to_velocity(img, z, t, eps: float):
    """JiTModel.image_to_velocity (src/models/jit/pipeline.py:253-260)."""
    return (img - z) / (1 - t.view(-1, 1, 1, 1)).clamp_min(eps)


def treat_loss(pred, z, x, t, loss_target: str = "image", t_eps: float = 0.05, model_pred: str = "image",
               noise=None):
    """JiTForClassToImageTraining.treat_loss: model_pred "image" (train/jit/arb_class_to_image.py:108-147) and
    model_pred "velocity" (train/jit/class_to_image.py:146-156: target clean - noise, no timestep clamp)."""
    if model_pred == "velocity":
        if loss_target != "velocity":
            raise NotImplementedError("Velocity prediction with image loss is not implemented yet.")
        return F.mse_loss(pred.float(), x.float() - noise.float())
    if loss_target == "image":
        return F.mse_loss(pred.float(), x.float())
    if loss_target == "velocity":
        return F.mse_loss(image_to_velocity(pred.float(), z, t, t_eps), image_to_velocity(x.float(), z, t, t_eps))
    raise ValueError(loss_target)


def class_tokenize(captions: list[str], label2id: dict[str, int], max_len: int, splitter: str = " "):
    """ClassTokenizer.tokenize (src/models/jit/class_encoder.py:42-90): ids padded with
    pad_id = len(label2id), mask 1 for real labels; unknown labels are skipped."""
    pad = len(label2id)
    ids, masks = [], []
    for text in captions:
        row = [label2id[s.strip()] for s in text.split(splitter) if s.strip() != "" and s.strip() in label2id]
        if len(row) < max_len:
            m = [1] * len(row) + [0] * (max_len - len(row))
            row = row + [pad] * (max_len - len(row))
        else:
            m, row = [1] * max_len, row[:max_len]
        ids.append(row)
        masks.append(m)
    return torch.tensor(ids, dtype=torch.long), torch.tensor(masks, dtype=torch.long)


def train_step_loss(model: OracleJiT, emb: torch.Tensor, batch: dict, loss_target: str = "image",
                    t_eps: float = 0.05, drop_context: bool = False, model_pred: str = "image", lowres_loss=()):
    """Forward half of train_step (train/jit/arb_class_to_image.py:153-276) with the random draws
    (t, noise) taken from `batch` and context ids already tokenised. lowres_loss: one more denoiser pass per
    scale on F.interpolate(mode="area") resized image / noisy image / noise, its loss added (arb:228-272).
    Returns (total loss, full-resolution pred)."""
    x = batch["image"].float()
    t = batch["t"]
    noise = batch["noise"].float()
    z = noised(x, t, noise)
    ids, mask = batch["ids"], batch["mask"]
    if drop_context:  # captions -> "" (all pad ids), mask -> ones (arb_class_to_image.py:162-189)
        ids = torch.full_like(ids, emb.shape[0] - 1)
        mask = torch.ones_like(mask)
    ctx = F.embedding(ids, emb, padding_idx=emb.shape[0] - 1)
    pred = model(z, t, ctx, batch["original_size"], batch["target_size"], batch["crop_coords"], mask)
    loss = treat_loss(pred, z, x, t, loss_target, t_eps, model_pred, noise)
    for s in lowres_loss:
        if s <= 0.0:  # arb:230-231
            continue

        def resize(v):  # arb:233-238
            return F.interpolate(v, scale_factor=s, mode="area")
        rx, rz = resize(x), resize(z)
        B, _, lh, lw = rx.shape
        size_lr = torch.tensor([[lh, lw]]).repeat(B, 1)
        pred_lr = model(rz, t, ctx, batch["original_size"] * s, size_lr, batch["crop_coords"] * s, mask)
        loss = loss + treat_loss(pred_lr, rz, rx, t, loss_target, t_eps, model_pred, resize(noise))
    return loss, pred


# ------------------------------------------------------------------------------- buckets
def generate_buckets(target_area: int = 1024 * 1024, start_size: int = 1024, step: int = 64,
                     min_size: int = 64) -> list[tuple[int, int]]:
    """src/dataset/aspect_ratio_bucket.py:20-60: (w, h) pairs of ~constant area."""
    out = []
    w = start_size
    while w >= min_size:
        h = round(target_area / w / step) * step
        if h < min_size:
            break
        out.append((w, h))
        if w != h:
            out.append((h, w))
        w -= step
    return out


def find_nearest_bucket(buckets: list[tuple[int, int]], width: int, height: int) -> int:
    """AspectRatioBucketManager.find_nearest (aspect_ratio_bucket.py:129-155)."""
    ar = math.log2(width / height)
    import numpy as np
    arr = np.array(buckets)
    order = np.argsort(-(arr[:, 0] * arr[:, 1]))  # same (unstable) order as the reference
    best, best_d = None, float("inf")
    for i in order:
        bw, bh = buckets[i]
        if bw > width or bh > height:
            continue
        d = abs(ar - math.log2(bw / bh))
        if d < best_d:
            best, best_d = i, d
    if best is None:
        raise AssertionError(f"No bucket found for image size {width}x{height}")
    return best


# ------------------------------------------------------------------------------- sampler
def generate(model: OracleJiT, emb: torch.Tensor, pos_ids: torch.Tensor, pos_mask: torch.Tensor,
             neg_ids: torch.Tensor, noise: torch.Tensor, num_inference_steps: int = 20, cfg_scale: float = 2.0,
             model_pred: str = "image", cfg_time_range=(0.0, 1.0)) -> torch.Tensor:
    """Euler sampler with classifier-free guidance -- JiTModel.generate (src/models/jit/pipeline.py:378-488)
    in execution dtype float32, class context. `noise` is the starting image (prepare_noisy_image,
    :124-148); timesteps = linspace(0, 1, steps + 1) (prepare_timesteps, :150-161); the negative prompts'
    embeddings are paired with the POSITIVE attention mask (prepare_context_embeddings, :193-219);
    size inputs (H, W) / (H, W) / (0, 0) (:221-248). Returns the final (clean) image, f32."""
    B, _, H, W = noise.shape
    do_cfg = cfg_scale > 1.0
    timesteps = torch.linspace(0.0, 1.0, num_inference_steps + 1)
    pad = emb.shape[0] - 1
    ctx_pos = F.embedding(pos_ids, emb, padding_idx=pad)
    ctx_neg = F.embedding(neg_ids, emb, padding_idx=pad)
    ctx = torch.cat([ctx_pos, ctx_neg]) if do_cfg else ctx_pos
    mask = torch.cat([pos_mask, pos_mask]) if do_cfg else pos_mask
    bb = 2 * B if do_cfg else B
    size = torch.tensor([[H, W]], dtype=torch.float32).repeat(bb, 1)
    crop = torch.zeros(bb, 2)
    z = noise.float().clone()
    for i, t in enumerate(timesteps[:-1]):
        in_cfg = do_cfg and cfg_time_range[0] <= float(t) <= cfg_time_range[1]   # pipeline.py:437-439
        x_in = torch.cat([z, z]) if in_cfg else z
        n = x_in.shape[0]
        pred = model(image=x_in, timestep=t.expand(n), context=ctx[:n], original_size=size[:n],
                     target_size=size[:n], crop_coords=crop[:n], context_mask=mask[:n])
        tb = t.expand(B).view(-1, 1, 1, 1)
        if model_pred == "image":                                               # :312-319, :340-353
            def to_v(img):
                return (img - z) / (1 - tb).clamp_min(1e-5)                     # image_to_velocity :254-260
        else:
            def to_v(v):
                return v
        if in_cfg:
            vp, vn = to_v(pred[:B]), to_v(pred[B:])
            v = vp + cfg_scale * (vp - vn)                                      # make_cfg_velocity_pred :351-357
        else:
            v = to_v(pred[:B])
        z = z + v * (timesteps[i + 1] - t)                                      # :477
    return z
