"""CPU ORACLE (test infrastructure only — never imported by the product path) for the SDXL QLoRA
rows of SURVEY §8(a): a29 LoRALinear over NF4 weights, a30 the SDXL TransformerBlock.

- TransformerBlock (src/models/sdxl/denoiser.py:208-280): LayerNorm -> SelfAttention (:30-98) ->
  LayerNorm -> CrossAttention (:101-171) -> LayerNorm -> FeedForward/GeGLU (:174-205), residuals.
- LoRALinear (src/modules/peft/lora.py:92-104): y = linear(x) + lora_up(lora_down(x)) * (alpha / rank).
- NF4 (bitsandbytes 0.48.2, not installed here; the reference wraps it in src/modules/quant/bnb.py:37-129):
  quant_type "nf4", blocksize 64, compress_statistics=True (nested absmax: offset = mean(absmax),
  8-bit blockwise quantisation of absmax - offset with blocksize 256 over bitsandbytes' signed dynamic
  map). Restated from bitsandbytes' published algorithm (functional.create_dynamic_map,
  quantize_4bit / dequantize_4bit, the NF4 code table); **parity unpinned** for the NF4 format itself
  (no bitsandbytes output exists here). Two nibbles per byte, the first element in the high nibble.

Parity of the block and of LoRA is pinned against fixtures produced by running the reference's own
TransformerBlock and LoRALinear (tests/golden/make_golden.py, sdxl_block.safetensors).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# bitsandbytes get_4bit_type("nf4"): quantiles of N(0,1) normalised to [-1, 1], 0 exact.
NF4 = torch.tensor([-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
                    -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
                    0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
                    0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0], dtype=torch.float32)


def dynamic_map(signed: bool = True, max_exponent_bits: int = 7, total_bits: int = 8) -> torch.Tensor:
    """bitsandbytes functional.create_dynamic_map (restated): 256 sorted values in [-1, 1]."""
    data = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    for i in range(max_exponent_bits):
        fraction_items = int(2 ** (i + non_sign_bits - max_exponent_bits) + 1 if signed
                             else 2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1)
        boundaries = torch.linspace(0.1, 1, fraction_items, dtype=torch.float32)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    if additional_items > 0:
        boundaries = torch.linspace(0.1, 1, additional_items + 1, dtype=torch.float32)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    data.append(0)
    data.append(1.0)
    data += [0] * (2 ** total_bits - len(data))
    data.sort()
    return torch.tensor(data, dtype=torch.float32)


def _nearest(x: torch.Tensor, code: torch.Tensor) -> torch.Tensor:
    """Index of the nearest code value (code sorted ascending), ties to the lower index."""
    d = (x.reshape(-1, 1) - code.reshape(1, -1)).abs()
    return d.argmin(dim=1)


def nf4_quantize(w: torch.Tensor, blocksize: int = 64, nested_blocksize: int = 256) -> dict[str, torch.Tensor]:
    """quantize_4bit(w, blocksize=64, compress_statistics=True, quant_type="nf4") restated.
    Returns packed uint8 [n/2], qabsmax uint8 [n/64], absmax2 f32 [ceil(n/64/256)], offset f32 [1],
    code2 f32 [256], shape."""
    flat = w.detach().float().reshape(-1)
    n = flat.numel()
    assert n % blocksize == 0 and n % 2 == 0
    blocks = flat.view(-1, blocksize)
    absmax = blocks.abs().amax(dim=1)
    scaled = blocks / absmax.clamp_min(1e-30).unsqueeze(1)
    q = _nearest(scaled, NF4).view(-1).to(torch.uint8)
    packed = (q[0::2] << 4) | q[1::2]
    offset = absmax.mean()
    a = absmax - offset
    nb2 = math.ceil(a.numel() / nested_blocksize)
    a_pad = torch.cat([a, torch.zeros(nb2 * nested_blocksize - a.numel())]).view(nb2, nested_blocksize)
    absmax2 = a_pad.abs().amax(dim=1)
    code2 = dynamic_map()
    q2 = _nearest(a_pad / absmax2.clamp_min(1e-30).unsqueeze(1), code2).view(-1)[: a.numel()].to(torch.uint8)
    return {"packed": packed, "qabsmax": q2, "absmax2": absmax2, "offset": offset.reshape(1), "code2": code2,
            "shape": torch.tensor(list(w.shape))}


def nf4_absmax(st: dict[str, torch.Tensor], blocksize: int = 64, nested_blocksize: int = 256) -> torch.Tensor:
    q2 = st["qabsmax"].long()
    blk2 = torch.arange(q2.numel()) // nested_blocksize
    return st["code2"][q2] * st["absmax2"][blk2] + st["offset"]


def nf4_dequantize(st: dict[str, torch.Tensor], blocksize: int = 64) -> torch.Tensor:
    """dequantize_4bit restated: W = NF4[code] * absmax[block] (f32), original shape."""
    p = st["packed"].long()
    codes = torch.stack([p >> 4, p & 15], dim=1).reshape(-1)
    absmax = nf4_absmax(st, blocksize)
    vals = NF4[codes] * absmax.repeat_interleave(blocksize)
    return vals.view(*[int(s) for s in st["shape"]])


# ---------------------------------------------------------------------------- TransformerBlock
LORA_TARGETS = ["attn1.to_q", "attn1.to_k", "attn1.to_v", "attn1.to_out.0", "attn2.to_q", "attn2.to_k",
                "attn2.to_v", "attn2.to_out.0", "ff.net.0.proj", "ff.net.2"]


def block_param_shapes(dim: int, heads: int, context_dim: int, rank: int, head_dim: int = 64):
    """Reference state-dict names/shapes of a TransformerBlock whose 10 Linear layers are wrapped by
    LoRALinear (`<target>.linear.weight|bias`, `<target>.lora_down.weight`, `<target>.lora_up.weight`)."""
    inner = heads * head_dim
    ffi = dim * 4
    lin = {"attn1.to_q": (inner, dim, False), "attn1.to_k": (inner, dim, False), "attn1.to_v": (inner, dim, False),
           "attn1.to_out.0": (dim, inner, True), "attn2.to_q": (inner, dim, False),
           "attn2.to_k": (inner, context_dim, False), "attn2.to_v": (inner, context_dim, False),
           "attn2.to_out.0": (dim, inner, True), "ff.net.0.proj": (2 * ffi, dim, True), "ff.net.2": (dim, ffi, True)}
    shapes = {}
    for t, (o, i, b) in lin.items():
        shapes[f"{t}.linear.weight"] = (o, i)
        if b:
            shapes[f"{t}.linear.bias"] = (o,)
        shapes[f"{t}.lora_down.weight"] = (rank, i)
        shapes[f"{t}.lora_up.weight"] = (o, rank)
    for k in ("norm1", "norm2", "norm3"):
        shapes[f"{k}.weight"] = (dim,)
        shapes[f"{k}.bias"] = (dim,)
    return shapes


def make_block_weights(dim, heads, context_dim, rank, seed, head_dim=64):
    g = torch.Generator().manual_seed(seed)
    w = {}
    for n, s in block_param_shapes(dim, heads, context_dim, rank, head_dim).items():
        if n.endswith("norm1.weight") or n.endswith("norm2.weight") or n.endswith("norm3.weight"):
            w[n] = 1.0 + 0.1 * torch.randn(s, generator=g)
        elif ".bias" in n or n.startswith("norm"):
            w[n] = 0.05 * torch.randn(s, generator=g)
        elif "lora_down" in n:
            w[n] = torch.randn(s, generator=g) / math.sqrt(s[1])
        elif "lora_up" in n:
            w[n] = 0.05 * torch.randn(s, generator=g)
        else:
            w[n] = torch.randn(s, generator=g) / math.sqrt(s[1])
    return w


def lora_linear(x, w, t, rank, alpha):
    """LoRALinear.forward (lora.py:92-104), dropout 0."""
    y = F.linear(x, w[f"{t}.linear.weight"], w.get(f"{t}.linear.bias"))
    return y + F.linear(F.linear(x, w[f"{t}.lora_down.weight"]), w[f"{t}.lora_up.weight"]) * (alpha / rank)


def block_forward(x, ctx, w, heads, rank, alpha, head_dim=64):
    """TransformerBlock.forward (denoiser.py:258-280) in fp32 with fp32 SDPA, LoRA on the 10 linears."""
    B, n, dim = x.shape
    nc = ctx.shape[1]

    def ln(h, k):
        return F.layer_norm(h, (dim,), w[f"{k}.weight"], w[f"{k}.bias"], eps=1e-5)

    def heads_of(t, L):
        return t.reshape(B, L, heads, head_dim).permute(0, 2, 1, 3)

    def attn(q, k, v, Lq):
        o = F.scaled_dot_product_attention(q, k, v)
        return o.permute(0, 2, 1, 3).reshape(B, Lq, heads * head_dim)

    h = ln(x, "norm1")
    q, k, v = (heads_of(lora_linear(h, w, f"attn1.to_{c}", rank, alpha), n) for c in "qkv")
    x = x + lora_linear(attn(q, k, v, n), w, "attn1.to_out.0", rank, alpha)
    h = ln(x, "norm2")
    q = heads_of(lora_linear(h, w, "attn2.to_q", rank, alpha), n)
    k = heads_of(lora_linear(ctx, w, "attn2.to_k", rank, alpha), nc)
    v = heads_of(lora_linear(ctx, w, "attn2.to_v", rank, alpha), nc)
    x = x + lora_linear(attn(q, k, v, n), w, "attn2.to_out.0", rank, alpha)
    h = ln(x, "norm3")
    hid, gate = lora_linear(h, w, "ff.net.0.proj", rank, alpha).chunk(2, dim=-1)     # GeGLU (:179-186)
    x = x + lora_linear(hid * F.gelu(gate), w, "ff.net.2", rank, alpha)
    return x


# ---------------------------------------------------------------------------- SpatialTransformer
def spatial_param_shapes(C: int, heads: int, depth: int, context_dim: int, rank: int, head_dim: int = 64):
    """Reference state-dict names/shapes of a SpatialTransformer (src/models/sdxl/denoiser.py:283-365) whose
    blocks' 10 Linear layers are LoRA-wrapped; norm = GroupNorm(32, C), proj_in / proj_out plain Linears."""
    inner = heads * head_dim
    shapes = {"norm.weight": (C,), "norm.bias": (C,), "proj_in.weight": (inner, C), "proj_in.bias": (inner,),
              "proj_out.weight": (C, inner), "proj_out.bias": (C,)}
    for i in range(depth):
        for n, s in block_param_shapes(inner, heads, context_dim, rank, head_dim).items():
            shapes[f"transformer_blocks.{i}.{n}"] = s
    return shapes


def make_spatial_weights(C, heads, depth, context_dim, rank, seed, head_dim=64):
    g = torch.Generator().manual_seed(seed)
    w = {}
    for n, s in spatial_param_shapes(C, heads, depth, context_dim, rank, head_dim).items():
        leaf = n.rsplit(".", 2)[-2] if n.count(".") >= 1 else n
        if n == "norm.weight" or n.endswith(("norm1.weight", "norm2.weight", "norm3.weight")):
            w[n] = 1.0 + 0.1 * torch.randn(s, generator=g)
        elif n.endswith(".bias"):
            w[n] = 0.05 * torch.randn(s, generator=g)
        elif "lora_down" in n:
            w[n] = torch.randn(s, generator=g) / math.sqrt(s[1])
        elif "lora_up" in n:
            w[n] = 0.05 * torch.randn(s, generator=g)
        else:
            w[n] = torch.randn(s, generator=g) / math.sqrt(s[1])
        del leaf
    return w


def spatial_forward(x, ctx, w, heads, depth, rank, alpha, head_dim=64, groups=32):
    """SpatialTransformer.forward (denoiser.py:331-365) in fp32: GroupNorm -> NCHW->tokens -> proj_in ->
    blocks -> proj_out -> tokens->NCHW -> + residual."""
    B, C, H, W = x.shape
    h = F.group_norm(x, groups, w["norm.weight"], w["norm.bias"], eps=1e-6)
    h = h.permute(0, 2, 3, 1).reshape(B, H * W, C)
    h = F.linear(h, w["proj_in.weight"], w["proj_in.bias"])
    for i in range(depth):
        pre = f"transformer_blocks.{i}."
        wb = {k[len(pre):]: v for k, v in w.items() if k.startswith(pre)}
        h = block_forward(h, ctx, wb, heads, rank, alpha, head_dim)
    h = F.linear(h, w["proj_out.weight"], w["proj_out.bias"])
    return h.reshape(B, H, W, C).permute(0, 3, 1, 2) + x


# ---------------------------------------------------------------------------- flow-matching step (config 5)
def sinusoid(t: torch.Tensor, dim: int, max_period: int = 10000) -> torch.Tensor:
    """get_timestep_embedding(t, dim, flip_sin_to_cos=True, downscale_freq_shift=0)
    (src/modules/timestep/embedding.py:10-62, called at src/models/sdxl/denoiser.py:1117-1123)."""
    half = dim // 2
    expo = -math.log(max_period) * torch.arange(0, half, dtype=torch.float32) / half
    emb = t[:, None].float() * torch.exp(expo)[None, :]
    return torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)


def flow_match_loss(latents, t, eps, ctx, pooled, sizes, sk, stacks, rank, alpha, noise_scale=1.0):
    """SDXLForFlowMatchingTraining.train_step (train/sdxl/flow_match.py:109-174) in fp32 on the skeleton UNet of
    vpt/sdxl_flow.py (the §8 transformer stacks, the reference's conditioning MLPs and emb_layers adds; frozen
    pixel-(un)shuffle + Linear maps in place of the conv / ResNet / resample path, skips as additions):
      z = t x + (1 - t) eps (prepare_scaled_noised_latents, flow_match.py:60-74), model timestep t * 1000,
      loss = mse(v, eps - x) (loss_with_predicted_velocity, flow_match.py:85-96).
    sk: the skeleton's weights {t1, t2, l1, l2, e_in, e_down, e_up, m_in, m_down, m_up, m_out} as (W, b|None);
    stacks: 11 (weights, heads, depth) in SDXL order (2 + 2 down, mid, 3 + 3 up)."""
    B, _, L, _ = latents.shape
    x = latents.float()
    tt = t.float().view(B, 1, 1, 1)
    z = tt * x + (1 - tt) * eps.float() * noise_scale

    def lin(name, h, bias=True):
        W, b = sk[name]
        return F.linear(h, W, b if bias else None)

    temb = lin("t2", F.silu(lin("t1", sinusoid(t * 1000.0, 320))))
    add = sinusoid(sizes.reshape(-1).float(), 256).reshape(B, -1)
    glob = lin("l2", F.silu(lin("l1", torch.cat([pooled.float(), add], 1)))) + temb
    sg = F.silu(glob)
    eA, eB, eU = lin("e_in", sg), lin("e_down", sg), lin("e_up", sg)

    def st(i, h):
        w, heads, depth = stacks[i]
        return spatial_forward(h, ctx, w, heads, depth, rank, alpha)

    def tok_lin(name, h, r, emb=None):
        """pixel_unshuffle(h, r) -> tokens -> Linear (+ per-sample emb) -> NCHW at the unshuffled size."""
        u = F.pixel_unshuffle(h, r) if r > 1 else h
        Bn, Cf, Hh, Ww = u.shape
        y = lin(name, u.permute(0, 2, 3, 1).reshape(Bn, Hh * Ww, Cf), bias=True)
        if emb is not None:
            y = y + emb[:, None, :]
        return y.reshape(Bn, Hh, Ww, -1).permute(0, 3, 1, 2)

    x64 = tok_lin("m_in", z, 2, eA)
    e0 = st(0, x64)
    e1 = st(1, e0)
    x32 = tok_lin("m_down", e1, 2, eB)
    d0 = st(2, x32)
    d1 = st(3, d0)
    m = st(4, d1)
    u0 = st(5, m + d1)
    u1 = st(6, u0 + d0)
    u2 = st(7, u1 + x32)
    y64 = F.pixel_shuffle(tok_lin("m_up", u2, 1, eU), 2)
    v0 = st(8, y64 + e1)
    v1 = st(9, v0 + e0)
    v2 = st(10, v1 + x64)
    v = F.pixel_shuffle(tok_lin("m_out", v2, 1), 2)
    return F.mse_loss(v, eps.float() * noise_scale - x), v
