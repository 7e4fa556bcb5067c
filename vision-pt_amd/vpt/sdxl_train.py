"""SDXL QLoRA step over the UNet's transformer stacks (BASELINE config 5).

The reference step is SDXLForFlowMatchingTraining.train_step (train/sdxl/flow_match.py:112-176) with the
config of configs/sdxl/flow_match/config.yml: NF4 (bitsandbytes) base weights, LoRA rank 16 / alpha 1.0 on
every `attn1`, `attn2` and `.ff.` Linear of the UNet's transformer blocks, batch 4, RAdamScheduleFree.
Its transformer part -- the 11 SpatialTransformers of the SDXL UNet (src/models/sdxl/denoiser.py:283-365,
placed by DownBlocks / MidBlock / UpBlocks :640-720, :800-815, :925-940) with their 70 TransformerBlocks,
700 LoRA targets -- is what this module runs, at the 1024^2 stage shapes (latent 128x128):

  stage        channels  heads  blocks/stack  tokens  stacks
  down 64x64      640      10        2         4096     2
  down 32x32     1280      20       10         1024     2
  mid  32x32     1280      20       10         1024     1
  up   32x32     1280      20       10         1024     3
  up   64x64      640      10        2         4096     3

with the text context of 3 x 77 = 231 tokens of width 2048 (CLIP-L | CLIP-G). Everything inside the stacks
runs on the HIP kernels (GroupNorm, NF4 dequant-in-GEMM with the LoRA term fused, LayerNorm, flash
attention self / cross, GeGLU, transposes, residuals in GEMM epilogues), the adapters' gradients land in one
flat f32 buffer and one fused RAdamScheduleFree launch steps them.

Not executed (outside SURVEY §8's rows): the UNet's ResNet / conv / up- and down-sampling path, the VAE
encoder and the text encoders. The stacks take synthetic stage activations as input and the step's loss is
sum_s <out_s, g_s> with fixed synthetic g_s (the gradient the UNet's remaining graph would hand back), so
every stack runs its full forward and backward (input, context and adapter gradients).
"""

from __future__ import annotations

import math

import torch

from . import ops
from .optim import RAdamScheduleFreeFlat
from .sdxl import TARGETS, SDXLSpatialTransformer, dynamic_map, lora_side_scope

BF16, F32 = torch.bfloat16, torch.float32

# (name, channels, heads, blocks per stack, latent side) at 1024^2 (latent 128x128)
SDXL_1024_STACKS = [("down.64.0", 640, 10, 2, 64), ("down.64.1", 640, 10, 2, 64),
                    ("down.32.0", 1280, 20, 10, 32), ("down.32.1", 1280, 20, 10, 32),
                    ("mid.32", 1280, 20, 10, 32),
                    ("up.32.0", 1280, 20, 10, 32), ("up.32.1", 1280, 20, 10, 32), ("up.32.2", 1280, 20, 10, 32),
                    ("up.64.0", 640, 10, 2, 64), ("up.64.1", 640, 10, 2, 64), ("up.64.2", 640, 10, 2, 64)]
CONTEXT_DIM = 2048
CONTEXT_TOKENS = 231


def _linear_shapes(dim: int, context_dim: int) -> dict[str, tuple[int, int]]:
    ffi = 4 * dim
    return {"attn1.to_q": (dim, dim), "attn1.to_k": (dim, dim), "attn1.to_v": (dim, dim), "attn1.to_out.0": (dim, dim),
            "attn2.to_q": (dim, dim), "attn2.to_k": (dim, context_dim), "attn2.to_v": (dim, context_dim),
            "attn2.to_out.0": (dim, dim), "ff.net.0.proj": (2 * ffi, dim), "ff.net.2": (dim, ffi)}


class SDXLStacksQLoRA:
    """The 11 SpatialTransformers with NF4 bases and LoRA adapters; adapters in one flat bf16 buffer (grads
    f32) stepped by RAdamScheduleFreeFlat. Synthetic random-init weights (no checkpoint is available here):
    bases N(0, 1/in) quantised to NF4 on the device, LoRA down kaiming-uniform and up zero as LoRALinear's
    init (src/modules/peft/lora.py:71-84), LayerNorm / GroupNorm weights 1, biases 0."""

    def __init__(self, B: int = 4, rank: int = 16, alpha: float = 1.0, stacks=SDXL_1024_STACKS,
                 context_dim: int = CONTEXT_DIM, n_ctx: int = CONTEXT_TOKENS, device="cuda", seed: int = 0,
                 lr: float = 1e-3):
        self.B, self.rank, self.alpha, self.n_ctx, self.cdim = B, rank, alpha, n_ctx, context_dim
        self.stacks_cfg = list(stacks)
        self.device = torch.device(device)
        g = torch.Generator(device=self.device).manual_seed(seed)
        # flat adapter layout, per stack and block: the downs of attn1.to_q / to_k / to_v side by side ([3r, in]:
        # the stacked B2 of the fused q|k|v input-gradient GEMM, vpt.sdxl), their ups, then every other target's
        # down [r, in] and up [out, r]
        # The cross-attention to_k / to_v adapters of ALL blocks live in three regions of their own (every down
        # [r, context_dim] side by side; the ups side by side per width class), so that precompute_ctx_kv runs the
        # k / v projections of the (fixed) text context for the whole step as stacked GEMMs.
        KV = ("attn2.to_k", "attn2.to_v")
        spans, total = [], 0
        for (_, C, heads, depth, _) in self.stacks_cfg:
            for _i in range(depth):
                shp = _linear_shapes(heads * 64, context_dim)
                qkv = ["attn1.to_q", "attn1.to_k", "attn1.to_v"]
                off = {t: [None, None] for t in KV}
                for t in qkv:
                    o, i = shp[t]
                    off[t] = [total, None]
                    total += rank * i
                for t in qkv:
                    o, i = shp[t]
                    off[t][1] = total
                    total += o * rank
                for t, (o, i) in shp.items():
                    if t not in off:
                        off[t] = [total, total + rank * i]
                        total += rank * i + o * rank
                for t, (o, i) in shp.items():
                    spans.append([off[t][0], (rank, i), off[t][1], (o, rank)])
        # the k / v regions: downs of every block, then the ups of the 1280-wide and of the 640-wide blocks
        widths = sorted({heads * 64 for (_, _, heads, _, _) in self.stacks_cfg}, reverse=True)
        # k / v targets by width class (1280 first), then in block order, k before v: the column order of the
        # step's ds = s * ctx . downs^T and of the stacked GEMM's output blocks
        kv_idx = sorted((k for k, _ in enumerate(spans) if TARGETS[k % len(TARGETS)] in KV),
                        key=lambda k: (-spans[k][3][0], k))
        self._kv_order = kv_idx
        self._kv_down0 = total
        for k in kv_idx:
            spans[k][0] = total
            total += rank * context_dim
        self._kv_up0 = {}
        for w in widths:
            self._kv_up0[w] = total
            for k in kv_idx:
                if spans[k][3][0] == w:
                    spans[k][2] = total
                    total += w * rank
        self.params = torch.zeros(total, dtype=BF16, device=self.device)
        self.grads = torch.zeros(total, dtype=F32, device=self.device)
        code2 = dynamic_map().to(self.device)
        self.stacks = []
        k = 0
        for (name, C, heads, depth, side) in self.stacks_cfg:
            dim = heads * 64
            sd = {"norm.weight": torch.ones(C, device=self.device), "norm.bias": torch.zeros(C, device=self.device),
                  "proj_in.weight": torch.randn(dim, C, device=self.device, generator=g) / math.sqrt(C),
                  "proj_in.bias": torch.zeros(dim, device=self.device),
                  "proj_out.weight": torch.randn(C, dim, device=self.device, generator=g) / math.sqrt(dim),
                  "proj_out.bias": torch.zeros(C, device=self.device)}
            for i in range(depth):
                pre = f"transformer_blocks.{i}."
                for t, (o, inf) in _linear_shapes(dim, context_dim).items():
                    d0, dsh, u0, ush = spans[k]
                    k += 1
                    down = self.params[d0:d0 + dsh[0] * dsh[1]].view(dsh)
                    down.copy_(((torch.rand(dsh, device=self.device, generator=g) * 2 - 1)
                                * math.sqrt(6.0 / inf)).to(BF16))
                    sd[pre + f"{t}.linear.weight"] = (torch.randn(o, inf, device=self.device, generator=g)
                                                      / math.sqrt(inf)).to(BF16)
                    if t in ("attn1.to_out.0", "attn2.to_out.0", "ff.net.0.proj", "ff.net.2"):
                        sd[pre + f"{t}.linear.bias"] = torch.zeros(o, device=self.device)
                    sd[pre + f"{t}.lora_down.weight"] = down
                    sd[pre + f"{t}.lora_up.weight"] = self.params[u0:u0 + ush[0] * ush[1]].view(ush)  # zeros
                for n in ("norm1", "norm2", "norm3"):
                    sd[pre + f"{n}.weight"] = torch.ones(dim, device=self.device)
                    sd[pre + f"{n}.bias"] = torch.zeros(dim, device=self.device)
            st = SDXLSpatialTransformer(C, heads, depth, context_dim, rank, alpha, sd, code2=code2, device=self.device)
            self.stacks.append((name, C, side * side, st))
            del sd
        # bind every adapter to its flat parameter / gradient slices (LoRALinearNF4 copies nothing: bf16 views)
        k = 0
        for (_, _, _, st) in self.stacks:
            for blk in st.blocks:
                for t in TARGETS:
                    d0, dsh, u0, ush = spans[k]
                    k += 1
                    lin = blk.lin[t]
                    lin.down = self.params[d0:d0 + dsh[0] * dsh[1]].view(dsh)
                    lin.up = self.params[u0:u0 + ush[0] * ush[1]].view(ush)
                    lin.g_down = self.grads[d0:d0 + dsh[0] * dsh[1]].view(dsh)
                    lin.g_up = self.grads[u0:u0 + ush[0] * ush[1]].view(ush)
        self.opt = RAdamScheduleFreeFlat(self.params, self.grads, lr=lr)
        self.opt.train()

    def n_adapter_params(self) -> int:
        return self.params.numel()

    def precompute_ctx_kv(self, ctx: torch.Tensor, save: bool = True) -> bool:
        """The cross-attention to_k / to_v of every block over the step's text context ctx [B*n_ctx, context_dim]:
        their bases dequantised (16 per launch), ds = s * ctx . [all k/v downs]^T as one GEMM, then one stacked
        base+LoRA GEMM per width class (vpt_gemm_bf16_lora_stacked). Each block's forward then takes its k / v column
        blocks (SDXLTransformerBlock.ctx_kv) and its adapters' backward the saved (ctx, ds) column slices. Returns
        False (nothing done: the blocks project per target) for the "inline" base mode or non-skinny adapters."""
        from .sdxl import _ctx_key, base_weight
        for (_, _, _, st) in self.stacks:
            for blk in st.blocks:
                blk.ctx_kv = None  # nothing from an earlier precompute survives this one
        all_lins = [blk.lin[t] for (_, _, _, st) in self.stacks for blk in st.blocks for t in TARGETS]
        owner = {id(blk.lin[t]): (blk, t) for (_, _, _, st) in self.stacks for blk in st.blocks for t in TARGETS}
        lins = [all_lins[k] for k in self._kv_order]
        if any(l.base_mode == "inline" or not (l.fused and l.skinny) for l in lins):
            return False
        if len({l.scale for l in lins}) != 1:
            return False  # one GEMM forms every target's ds with one LoRA scale: only when they all share it
        key = _ctx_key(ctx)
        r, cd, M = self.rank, self.cdim, ctx.shape[0]
        downs = self.params[self._kv_down0:self._kv_down0 + len(lins) * r * cd].view(len(lins) * r, cd)
        ds = torch.empty(M, len(lins) * r, dtype=BF16, device=self.device)
        ops.gemm(ctx, True, downs, True, M, len(lins) * r, cd, ds, alpha=lins[0].scale)
        c0 = 0
        for w, u0 in self._kv_up0.items():
            group = [l for l in lins if l.base.shape[0] == w]
            G = len(group)
            ups = self.params[u0:u0 + G * w * r].view(G * w, r)
            if group[0].base_mode == "resident":
                W = self._kv_resident.get(w) if hasattr(self, "_kv_resident") else None
                if W is None:
                    W = torch.cat([base_weight(l.base, "resident", self.device) for l in group], 0)
                    self._kv_resident = {**getattr(self, "_kv_resident", {}), w: W}
            else:
                W = ops.workspace(self.device, f"kv_base{w}", G * w * cd, BF16).view(G * w, cd)
                ops.nf4_dequant_batch([(l.base, W[i * w:(i + 1) * w]) for i, l in enumerate(group)])
            out = ops.workspace(self.device, f"kv_out{w}", M * G * w, BF16).view(M, G * w)
            ops.gemm_lora_stacked(ctx, W, ds[:, c0:c0 + G * r], ups, w, out)
            for i, l in enumerate(group):
                l._saved = (ctx, ds[:, c0 + i * r:c0 + (i + 1) * r]) if save else None
                blk, t = owner[id(l)]
                kv = list(blk.ctx_kv or (None, None, key))
                kv[0 if t == "attn2.to_k" else 1] = out[:, i * w:(i + 1) * w]
                blk.ctx_kv = tuple(kv)
            c0 += G * r
        return True

    def make_inputs(self, seed: int = 1, hws=None):
        """Synthetic stage activations (NCHW bf16), text context [B*231, 2048] and output gradients g_s. hws: the
        token count of each stack (an aspect-ratio bucket's stage h x w); default the configured square sides."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        hws = [HW for (_, _, HW, _) in self.stacks] if hws is None else list(hws)
        xs = [torch.randn(self.B, C, hw, device=self.device, generator=g).to(BF16)
              for (_, C, _, _), hw in zip(self.stacks, hws)]
        gs = [(torch.randn(self.B, C, hw, device=self.device, generator=g) * 1e-3).to(BF16)
              for (_, C, _, _), hw in zip(self.stacks, hws)]
        ctx = torch.randn(self.B * self.n_ctx, self.cdim, device=self.device, generator=g).to(BF16)
        return xs, ctx, gs

    def step(self, xs, ctx, gs):
        """One training step: forward of every stack, backward in reverse order, fused optimizer step. Each
        stack's token count is its input's (xs[i] [B, C, HW]: any bucket). Returns the context gradient (summed
        over stacks), [B*231, 2048] bf16."""
        self.grads.zero_()
        self.precompute_ctx_kv(ctx)
        for x, (_, C, _, st) in zip(xs, self.stacks):
            st.forward(x, ctx, self.B, x.shape[2], self.n_ctx)
        dctx = None
        with lora_side_scope(self.device):  # adapter gradients beside the chain, joined before the optimizer
            for gout, (_, C, _, st) in zip(reversed(gs), reversed(self.stacks)):
                _dx, dc = st.backward(gout)
                dctx = dc if dctx is None else ops.add_bf16(dctx, dc)
        self.opt.step()
        return dctx

    def flops_per_step(self, hws=None) -> float:
        """Algorithmic FLOPs of one step: forward + backward of every GEMM (QLoRA: no base-weight gradient;
        LoRA down/up forward, their weight and input gradients) and attention (backward = 2x forward). hws: each
        stack's token count (default the configured square sides)."""
        B, r, nc, cd = self.B, self.rank, self.n_ctx, self.cdim
        f = 0.0
        hws = [HW for (_, _, HW, _) in self.stacks] if hws is None else list(hws)
        for (_, C, _, st), HW in zip(self.stacks, hws):
            M = B * HW
            dim = st.inner
            f += 2 * (2 * M * C * dim)            # proj_in / proj_out forward
            f += 2 * (2 * M * C * dim)            # their input gradients
            for _ in st.blocks:
                for t, (o, i) in _linear_shapes(dim, cd).items():
                    m = B * nc if t in ("attn2.to_k", "attn2.to_v") else M
                    f += 2 * m * o * i + 2 * m * r * (i + o)          # base + LoRA forward
                    f += 2 * m * o * i + 2 * (2 * m * r * (i + o))    # input grad + LoRA grads
                heads = st.heads
                f += 3 * 4 * B * heads * HW * HW * 64                 # self-attention fwd + bwd
                f += 3 * 4 * B * heads * HW * nc * 64                 # cross-attention fwd + bwd
        return f
