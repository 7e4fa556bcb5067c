"""SDXL QLoRA rows of SURVEY §8(a) on the HIP kernels:

a29  LoRALinearNF4: LoRALinear (src/modules/peft/lora.py:92-104) over a bitsandbytes NF4 Linear4bit
     (src/modules/quant/bnb.py:37-129): y = bf16(bf16(x W^T + b) + bf16(s * up(down(x)))), s = alpha/rank,
     the LoRA term fused into the base GEMM as a K-extension (one f32 accumulator), the NF4 base entering it
     as BASE_MODES below says (default: dequantised per call as bitsandbytes' MatMul4Bit does). Base weight
     frozen; the adapters train (f32 grads).
a30  SDXLTransformerBlock: TransformerBlock.forward (src/models/sdxl/denoiser.py:258-280) --
     LayerNorm -> self-attention -> LayerNorm -> cross-attention to the text context -> LayerNorm ->
     GeGLU feed-forward, residuals -- with its 10 Linear layers as LoRALinearNF4 (the QLoRA targets),
     forward with saved activations and the backward of the reference's bf16 autograd graph (grads of
     the input, the context and every adapter).
"""

from __future__ import annotations


import contextlib

import torch

from . import ops

BF16 = torch.bfloat16
F32 = torch.float32
U8 = torch.uint8


def dynamic_map(signed: bool = True, max_exponent_bits: int = 7, total_bits: int = 8) -> torch.Tensor:
    """bitsandbytes functional.create_dynamic_map (0.48.2): the 256-value signed map the nested absmax
    statistics are quantised over (quantize_4bit(..., compress_statistics=True)); sorted, in [-1, 1]."""
    data = []
    non_sign = total_bits - 1
    extra = 2 ** (non_sign - max_exponent_bits) - 1
    for i in range(max_exponent_bits):
        n = int(2 ** (i + non_sign - max_exponent_bits) + 1 if signed else 2 ** (i + non_sign - max_exponent_bits + 1) + 1)
        bnd = torch.linspace(0.1, 1, n, dtype=torch.float32)
        mid = (bnd[:-1] + bnd[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * mid).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * mid).tolist()
    if extra > 0:
        bnd = torch.linspace(0.1, 1, extra + 1, dtype=torch.float32)
        mid = (bnd[:-1] + bnd[1:]) / 2.0
        data += ((10 ** (-(max_exponent_bits - 1) + i)) * mid).tolist()
        if signed:
            data += (-(10 ** (-(max_exponent_bits - 1) + i)) * mid).tolist()
    data += [0, 1.0]
    data += [0] * (2 ** total_bits - len(data))
    data.sort()
    return torch.tensor(data, dtype=torch.float32)


class NF4Weight:
    """Device-resident NF4 tensor in the bitsandbytes layout (see include/vpt_hip.h)."""

    def __init__(self, packed, qabsmax, absmax2, code2, offset, shape):
        self.packed, self.qabsmax, self.absmax2, self.code2, self.offset = packed, qabsmax, absmax2, code2, offset
        self.resident = None  # bf16 base of the "resident" mode (built on first use)
        self.resident_qkv = None  # "resident" mode, attn1.to_q only: the stacked q|k|v bases
        self.shape = tuple(int(s) for s in shape)
        self.numel = 1
        for s in self.shape:
            self.numel *= s

    @classmethod
    def from_state(cls, st: dict[str, torch.Tensor], device="cuda"):
        """From {packed, qabsmax, absmax2, code2, offset, shape} (the bnb quant_state fields)."""
        d = {k: v.to(device) for k, v in st.items() if k != "shape"}
        return cls(d["packed"].to(U8).contiguous(), d["qabsmax"].to(U8).contiguous(), d["absmax2"].float().contiguous(),
                   d["code2"].float().contiguous(), d["offset"].float().reshape(1).contiguous(), st["shape"].tolist())

    @classmethod
    def quantize(cls, w: torch.Tensor, code2: torch.Tensor):
        """quantize_4bit(w, blocksize=64, compress_statistics=True, quant_type="nf4") on the device."""
        w = w.to(BF16).contiguous()
        n = w.numel()
        dev = w.device
        packed = torch.empty(n // 2, dtype=U8, device=dev)
        qabsmax = torch.empty(n // 64, dtype=U8, device=dev)
        absmax2 = torch.empty((n // 64 + 255) // 256, dtype=F32, device=dev)
        offset = torch.empty(1, dtype=F32, device=dev)
        scratch = torch.empty(n // 64, dtype=F32, device=dev)
        code2 = code2.to(dev, F32).contiguous()
        ops.nf4_quantize(w, code2, packed, qabsmax, absmax2, offset, scratch)
        return cls(packed, qabsmax, absmax2, code2, offset, w.shape)

    def dequantize(self, out: torch.Tensor | None = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.shape, dtype=BF16, device=self.packed.device)
        return ops.nf4_dequant(self.packed, self.qabsmax, self.absmax2, self.code2, self.offset, self.numel,
                               out.view(self.shape))


# How the frozen NF4 base enters the GEMM (BASELINE config 5):
#   "dequant"  (default) bitsandbytes' MatMul4Bit semantics (bnb 0.48.2 matmul_4bit for a multi-row input:
#              dequantize_4bit(W) to a bf16 weight, then F.linear; its backward dequantises again): each forward and
#              each input-gradient call dequantises W (vpt_nf4_dequant, 16-B vectorised, HBM-bound) into one
#              per-device scratch and runs the bf16 ring / T128 GEMM with the LoRA term as a K-extension
#              (vpt_gemm_bf16_lora). Only the NF4 state stays resident.
#   "resident" the dequantised bf16 base kept in HBM next to its NF4 state (frozen, so it is computed once; 4.4 GB
#              for the SDXL UNet's transformer Linears -- room the 288 GB of an MI355X has), same GEMMs.
#   "inline"   NF4 dequantised tile by tile inside the GEMM (vpt_gemm_nf4: no bf16 weight in HBM at all; the
#              memory-lean variant, ~1.5x slower on the config-5 shapes).
# All three give the same dequantised values; "dequant" and "resident" give bitwise identical outputs.
BASE_MODES = ("dequant", "resident", "inline")
DEFAULT_BASE_MODE = "dequant"
_SCRATCH: dict = {}  # (device, "call" | "block") -> bf16 dequant scratch, grown on demand


def _dequant_scratch(base: "NF4Weight", device) -> torch.Tensor:
    buf = _SCRATCH.get((str(device), "call"))
    if buf is None or buf.numel() < base.numel:
        buf = _SCRATCH[(str(device), "call")] = torch.empty(base.numel, dtype=BF16, device=device)
    return base.dequantize(buf[:base.numel].view(base.shape))


def dequant_bases(lins: dict, targets, device) -> dict:
    """{target: bf16 base} for a block's LoRA targets about to run: "dequant" mode dequantises all of them in ONE
    launch (vpt_nf4_dequant_batch) into a shared per-device scratch (stream-ordered reuse, block after block);
    "resident" returns the kept bf16 bases; "inline" (or a non-fused target) returns nothing (the GEMM dequantises)."""
    ts = [t for t in targets if lins[t].fused and lins[t].base_mode != "inline"]
    if not ts:
        return {}
    if lins[ts[0]].base_mode == "resident":
        out = {t: base_weight(lins[t].base, "resident", device) for t in ts}
        if ts[:3] == QKV:
            q = lins[QKV[0]].base
            if q.resident_qkv is None:  # the stacked copy of the fused q|k|v GEMMs, kept with the q base
                q.resident_qkv = torch.cat([out[t] for t in QKV], 0)
            out["attn1.qkv"] = q.resident_qkv
        return out
    total = sum(lins[t].base.numel for t in ts)
    buf = _SCRATCH.get((str(device), "block"))
    if buf is None or buf.numel() < total:
        buf = _SCRATCH[(str(device), "block")] = torch.empty(total, dtype=BF16, device=device)
    out, off = {}, 0
    for t in ts:
        b = lins[t].base
        out[t] = buf[off:off + b.numel].view(b.shape)
        off += b.numel
    ops.nf4_dequant_batch([(lins[t].base, out[t]) for t in ts])
    if ts[:3] == QKV:  # the three self-attention bases are side by side: the stacked [3 dim, dim] operand
        n = lins[QKV[0]].base.numel
        out["attn1.qkv"] = buf[:3 * n].view(3 * lins[QKV[0]].base.shape[0], lins[QKV[0]].base.shape[1])
    return out


def base_weight(base: "NF4Weight", mode: str, device) -> torch.Tensor:
    """The bf16 base weight a "dequant" / "resident" GEMM reads (stream-ordered scratch reuse for "dequant")."""
    if mode == "resident":
        if base.resident is None:
            base.resident = base.dequantize()
        return base.resident
    return _dequant_scratch(base, device)


class LoRALinearNF4:
    """a29. `down` [r, in], `up` [out, r] bf16 trainable (grads `g_down`, `g_up` f32); `base` NF4 [out, in].

    forward  ds = bf16(s * x . down^T)            (one skinny GEMM, s = alpha / rank folded into its epilogue)
             y  = bf16(x . Wd^T + b + ds . up^T)  (vpt_gemm_bf16_lora on the dequantised base, or vpt_gemm_nf4
                                                   in "inline" mode: LoRA term as K-extension, no LoRA add pass)
    backward g_up += dy^T . ds;  vs = bf16(s * dy . up);  g_down += vs^T . x;
             dx = bf16(dy . Wd + vs . down)       (the same two GEMMs in the input-gradient direction)
    The reference (lora.py:92-104) rounds lora_down, lora_up and their scaled sum to bf16 separately; here the
    sum is taken in f32 before one rounding (within the bf16 parity tolerance of tests/test_sdxl_gpu.py)."""

    def __init__(self, base: NF4Weight, bias: torch.Tensor | None, down: torch.Tensor, up: torch.Tensor,
                 alpha: float, rank: int, base_mode: str | None = None):
        self.base, self.bias = base, bias
        self.base_mode = base_mode or DEFAULT_BASE_MODE
        if self.base_mode not in BASE_MODES:
            raise ValueError(f"base_mode must be one of {BASE_MODES}")
        self.down, self.up = down.to(BF16).contiguous(), up.to(BF16).contiguous()
        self.scale = alpha / rank
        self.g_down = torch.zeros(self.down.shape, dtype=F32, device=self.down.device)
        self.g_up = torch.zeros(self.up.shape, dtype=F32, device=self.up.device)
        self._saved = None
        # NF4 blocks (64 elements of the flat [out][in] weight) must not straddle rows for the per-tile
        # dequant: true for every SDXL UNet Linear (in/out features are multiples of 64); other shapes take
        # the dequant-to-scratch path below.
        self.fused = base.shape[0] % 64 == 0 and base.shape[1] % 64 == 0
        # rank-16 skinny kernels (vpt_lora_proj / vpt_lora_wgrad) where the widths allow; generic GEMMs otherwise
        self.skinny = rank == 16 and self.down.shape[0] == 16 and base.shape[0] % 128 == 0 and base.shape[1] % 128 == 0

    def weight(self) -> torch.Tensor:
        """The dequantised base weight (bf16) -- for tests and export only; the hot path never builds it."""
        return self.base.dequantize(torch.empty(self.base.shape, dtype=BF16, device=self.down.device))

    def forward(self, x: torch.Tensor, save: bool = True, out: torch.Tensor | None = None,
                resid: torch.Tensor | None = None, W: torch.Tensor | None = None,
                ds: torch.Tensor | None = None, out_scale: float = 1.0) -> torch.Tensor:
        """resid: a bf16 tensor added in the epilogue (the block's residual stream: bf16(resid + bf16(y))).
        W: the base already dequantised by the caller (dequant_bases), else this call dequantises it.
        ds: s * x . down^T already computed by the caller (the fused LayerNorm, ops.layernorm_lora_fwd).
        out_scale: y = bf16(out_scale * (x . Wd^T + ds . up^T)) -- the attention q emitted pre-scaled (a Linear
        without bias or residual); folded into the GEMM epilogue on the dequant and inline paths."""
        if out_scale != 1.0 and (self.bias is not None or resid is not None):
            raise ValueError("out_scale: a Linear without bias / residual only")
        M = x.shape[0]
        r = self.down.shape[0]
        if ds is not None:
            pass
        elif self.skinny:
            ds = torch.empty(M, r, dtype=BF16, device=x.device)
            ops.lora_proj(x, self.down, True, ds, alpha=self.scale)
        else:
            ds = torch.empty(M, r, dtype=BF16, device=x.device)
            ops.gemm(x, True, self.down, True, M, r, x.shape[1], ds, alpha=self.scale)
        y = out if out is not None else torch.empty(M, self.base.shape[0], dtype=BF16, device=x.device)
        if self.fused and self.base_mode != "inline":
            W = base_weight(self.base, self.base_mode, x.device) if W is None else W
            ops.gemm_lora(x, W, True, ds, self.up, M, W.shape[0], W.shape[1], y, bias=self.bias, resid=resid,
                          alpha=out_scale)
        elif self.fused:
            ops.gemm_nf4(x, self.base, True, y, lora_a=ds, lora_b=self.up, bias=self.bias, resid=resid, alpha=out_scale)
        else:
            lo = ops.gemm(ds, True, self.up, True, M, self.up.shape[0], r,
                          torch.empty(M, self.up.shape[0], dtype=BF16, device=x.device))
            ops.linear(x, self.weight(), bias=self.bias, resid=lo, out=y)
            if resid is not None:
                y = ops.add_bf16(resid, y)
            if out_scale != 1.0:
                y = ops.scale_bf16(y, out_scale)
        self._saved = (x, ds) if save else None
        return y

    def backward(self, dy: torch.Tensor, need_dx: bool = True, W: torch.Tensor | None = None,
                 vs: torch.Tensor | None = None) -> torch.Tensor | None:
        """Accumulates g_up, g_down; returns dx (bf16), or None with need_dx=False (an input that needs no
        gradient, e.g. the frozen text encoder's hidden states under attn2.to_k / to_v). vs: s * dy . up already
        computed by the caller (ops.lora_proj_grouped over adjacent targets)."""
        vs = self.backward_adapters(dy, vs_out=vs, vs_ready=vs is not None)
        if not need_dx:
            return None
        x = self._saved[0]
        M = x.shape[0]
        dx = torch.empty(M, self.base.shape[1], dtype=BF16, device=dy.device)
        if self.fused and self.base_mode != "inline":
            W = base_weight(self.base, self.base_mode, dy.device) if W is None else W
            return ops.gemm_lora(dy, W, False, vs, self.down, M, W.shape[1], W.shape[0], dx)
        if self.fused:
            return ops.gemm_nf4(dy, self.base, False, dx, lora_a=vs, lora_b=self.down)
        dx_lora = ops.linear_dgrad(vs, self.down)
        return ops.linear_dgrad(dy, self.weight(), resid=dx_lora, out=dx)

    def backward_adapters(self, dy: torch.Tensor, vs_out: torch.Tensor | None = None,
                          vs_ready: bool = False) -> torch.Tensor:
        """The adapter half of the backward: g_up += dy^T . ds, vs = bf16(s * dy . up), g_down += vs^T . x;
        returns vs (into vs_out when given: a column block of a fused q|k|v gradient's LoRA operand; vs_ready: the
        caller already wrote vs there, ops.lora_proj_grouped)."""
        x, ds = self._saved
        M = x.shape[0]
        r = self.down.shape[0]
        vs = torch.empty(M, r, dtype=BF16, device=dy.device) if vs_out is None else vs_out
        if self.skinny:
            if not vs_ready:
                ops.lora_proj(dy, self.up, False, vs, alpha=self.scale)
            ops.lora_wgrad2(dy, ds, self.g_up, x, vs, self.g_down)
        else:
            ops.linear_wgrad(dy, ds, self.g_up, accumulate=True, splits=ops.wgrad_splits(*self.up.shape, M))
            ops.gemm(dy, True, self.up, False, M, r, self.up.shape[0], vs, alpha=self.scale)
            ops.linear_wgrad(vs, x, self.g_down, accumulate=True, splits=ops.wgrad_splits(*self.down.shape, M))
        return vs


# Module attributes (tools/c5_knob_ab.py assigns them in-process for A/B runs; no environment switches).
# False = LayerNorm (forward / backward) and the LoRA projections of its output as separate launches
FUSED_LN_LORA = True
FUSED_LN_BWD_LORA = True  # the backward half alone
# True = the attention q projections emit q * scale * log2(e) from their GEMM epilogue (one rounding);
# False = a bf16 q, then a separate scaling pass (two roundings, one more launch per q)
FOLD_Q_SCALE = True
# True = the GeGLU backward also emits ff.net.0.proj's input-gradient LoRA operand (ops.geglu_bwd_lora)
FUSED_GEGLU_LORA = True
# True = the GeGLU forward also emits ff.net.2's LoRA down-projection (ops.geglu_fwd_lora)
FUSED_GEGLU_LORA_FWD = True
# True = a transformer block's norm1 backward also emits the input-gradient LoRA operand of the previous block's
# ff.net.2 (whose output gradient that dx is; ops.layernorm_bwd_lora, bit-identical to the separate lora_proj)
FUSED_LN_BWD_PREV = True
# True = inside a training step's backward (lora_side_scope), each block's batched adapter-gradient launches
# (ops.lora_wgrad_batch) run on a side stream beside the input-gradient chain (nothing in the chain reads an adapter
# gradient); the scope's exit joins the side stream, before anything reads the adapter gradients. Measured -1.5 % per
# C5 step (r05zm: the batched slab / reduce launches are short and their join points close), so off.
LORA_WGRAD_SIDE = False
_SIDE: dict = {}
_SIDE_SCOPE = [0]


def lora_side(device) -> torch.cuda.Stream | None:
    """The adapter-gradient side stream of a device while a lora_side_scope is open (else None: same stream)."""
    if not (LORA_WGRAD_SIDE and _SIDE_SCOPE[0]) or torch.device(device).type != "cuda":
        return None
    key = str(torch.device(device))
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


@contextlib.contextmanager
def lora_side_scope(device):
    """A training step's backward: adapter-gradient batches on the side stream; on exit the caller's stream waits
    for all of them (the adapter gradients are then complete in its order)."""
    _SIDE_SCOPE[0] += 1
    try:
        yield
    finally:
        _SIDE_SCOPE[0] -= 1
        st = _SIDE.get(str(torch.device(device)))
        if st is not None:
            torch.cuda.current_stream(device).wait_stream(st)


def _ctx_key(ctx: torch.Tensor) -> tuple:
    """Identity of a context tensor for SDXLTransformerBlock.ctx_kv (storage address, shape, strides, version)."""
    return (ctx.data_ptr(), tuple(ctx.shape), tuple(ctx.stride()), ctx._version)


def _adjacent(ts) -> bool:
    """Contiguous tensors laid out back to back (the flat adapter layout of SDXLStacksQLoRA)."""
    return all(t.is_contiguous() for t in ts) and all(
        ts[i].data_ptr() + ts[i].numel() * ts[i].element_size() == ts[i + 1].data_ptr() for i in range(len(ts) - 1))


TARGETS = ["attn1.to_q", "attn1.to_k", "attn1.to_v", "attn1.to_out.0", "attn2.to_q", "attn2.to_k", "attn2.to_v",
           "attn2.to_out.0", "ff.net.0.proj", "ff.net.2"]
QKV = TARGETS[:3]


class SDXLTransformerBlock:
    """a30. Weights from a reference-named state dict: `<target>.linear.weight` given either as an NF4
    state ({packed, qabsmax, absmax2, code2, offset, shape}) or as a dense tensor (quantised on load),
    `<target>.linear.bias`, `<target>.lora_down.weight`, `<target>.lora_up.weight`, `norm{1,2,3}.{weight,bias}`."""

    def __init__(self, dim: int, heads: int, context_dim: int, rank: int, alpha: float, sd: dict, code2=None,
                 device="cuda", head_dim: int = 64):
        if head_dim != 64:
            raise NotImplementedError("attention kernels are head_dim 64 (SDXL: 64)")
        self.dim, self.heads, self.cdim, self.rank = dim, heads, context_dim, rank
        self.inner = heads * 64
        self.device = device
        self.lin = {}
        for t in TARGETS:
            base = _nf4_or_dense(sd[f"{t}.linear.weight"], code2, device)
            b = sd.get(f"{t}.linear.bias")
            self.lin[t] = LoRALinearNF4(base, None if b is None else b.to(device, BF16).contiguous(),
                                        sd[f"{t}.lora_down.weight"].to(device), sd[f"{t}.lora_up.weight"].to(device),
                                        alpha, rank)
        self.norm = {k: (sd[f"{k}.weight"].to(device, BF16).contiguous(), sd[f"{k}.bias"].to(device, BF16).contiguous())
                     for k in ("norm1", "norm2", "norm3")}
        self._st = None
        self.vs_prev = None  # the previous block's ff.net.2 vs from the last backward (backward(prev_ff2=...))
        # (k, v, ctx key) of the cross-attention, projected for the next forward by the caller (SDXLStacksQLoRA.
        # precompute_ctx_kv: every block's over one fixed context in stacked GEMMs); used only by a forward over
        # the context it was projected from (_ctx_key); None: projected here
        self.ctx_kv = None

    def _attn_fwd(self, q, k, v, B, n, nk):
        """q must already be pre-scaled (`_qs`); the backward returns the gradient of the raw q."""
        o = torch.empty(B * n, self.inner, dtype=BF16, device=self.device)
        lse = torch.empty(B, self.heads, n, dtype=F32, device=self.device)
        H = self.heads
        ops.attn_fwd(ops._t4(q, B, n, H), ops._t4(k, B, nk, H), ops._t4(v, B, nk, H), ops._t4(o, B, n, H), lse, None,
                     B, H, n, n, nk, nk=nk)
        return o, lse

    @staticmethod
    def _q_out_scale() -> float:
        """The q projections' output scale when it is folded into their GEMM epilogue (FOLD_Q_SCALE), else 1."""
        return ops.attn_q_scale(0.125) if FOLD_Q_SCALE else 1.0

    @staticmethod
    def _qs(q):
        """The attention kernels take q pre-multiplied by scale*log2(e) (include/vpt_hip.h)."""
        return ops.scale_bf16(q, ops.attn_q_scale(0.125))

    def _fuse_qkv(self, Wb: dict) -> bool:
        """The self-attention q / k / v projections run as one GEMM each way when their bases are stacked
        (dequant_bases) and their adapters take the rank-16 skinny kernels."""
        return "attn1.qkv" in Wb and all(self.lin[t].skinny for t in QKV)

    def _ln_lora(self, x, norm: str, targets) -> tuple:
        """LayerNorm `norm` of x and the LoRA down-projections of its output for `targets` (adjacent downs, one
        scale, rank-16 skinny) in one launch (ops.layernorm_lora_fwd): (y, mean, rstd, ds [M, 16 len(targets)]);
        ds None where the fused form does not apply (the projections then run in LoRALinearNF4.forward)."""
        L = self.lin
        downs = [L[t].down for t in targets]
        if FUSED_LN_LORA and all(L[t].skinny for t in targets) and _adjacent(downs) \
                and len({L[t].scale for t in targets}) == 1 and x.shape[1] % 128 == 0:
            ds = torch.empty(x.shape[0], 16 * len(targets), dtype=BF16, device=x.device)
            y, m, r = ops.layernorm_lora_fwd(x, *self.norm[norm], downs[0], len(targets), L[targets[0]].scale, ds)
            return y, m, r, ds
        return (*ops.layernorm_fwd(x, *self.norm[norm]), None)

    def _ln_bwd_lora(self, dy, x, mean, rstd, norm: str, dres, target):
        """LayerNorm backward of `norm` and the input-gradient LoRA operand vs = s * dx . up of `target` (the
        LoRALinear that consumes dx as its output gradient: a name in this block, or the LoRALinear itself) in one
        launch (ops.layernorm_bwd_lora): (dx, vs); vs None where the fused form does not apply."""
        lin = self.lin[target] if isinstance(target, str) else target
        if FUSED_LN_LORA and FUSED_LN_BWD_LORA and lin.skinny and lin.up.is_contiguous() and x.shape[1] % 128 == 0:
            vs = torch.empty(x.shape[0], 16, dtype=BF16, device=x.device)
            dx = ops.layernorm_bwd_lora(dy, x, mean, rstd, self.norm[norm][0], lin.up, lin.scale, vs, dres=dres)
            return dx, vs
        return ops.layernorm_bwd(dy, x, mean, rstd, self.norm[norm][0], dres=dres), None

    def _qkv_fwd(self, h1, Wqkv, save, ds=None):
        """q|k|v = h1 . [Wq; Wk; Wv]^T + [ds_q | ds_k | ds_v] . blockdiag(up_q, up_k, up_v)^T as ONE GEMM
        (vpt_gemm_bf16_lora_grouped; each output column block is exactly its target's LoRALinear), q pre-scaled for
        the attention kernels in the same epilogue (FOLD_Q_SCALE; else in place afterwards). Returns column views (q, k, v) of the [M, 3 dim] output."""
        M, D, L = h1.shape[0], self.inner, self.lin
        r = L[QKV[0]].down.shape[0]
        downs = [L[t].down for t in QKV]
        grouped = _adjacent(downs) and len({L[t].scale for t in QKV}) == 1
        if ds is not None:  # computed with the LayerNorm (ops.layernorm_lora_fwd)
            grouped = True
        elif grouped:  # the flat layout: ds_q | ds_k | ds_v in one launch
            ds = torch.empty(M, 3 * r, dtype=BF16, device=h1.device)
            ops.lora_proj_grouped(h1, 0, downs[0], downs[0].numel(), 3, True, ds, alpha=L[QKV[0]].scale)
        else:
            ds = torch.empty(M, 3 * r, dtype=BF16, device=h1.device)
        for g, t in enumerate(QKV):
            dsg = ds[:, g * r:(g + 1) * r]
            if not grouped:
                ops.lora_proj(h1, L[t].down, True, dsg, alpha=L[t].scale)
            L[t]._saved = (h1, dsg) if save else None
        qkv = torch.empty(M, 3 * D, dtype=BF16, device=h1.device)
        if FOLD_Q_SCALE:
            ops.gemm_lora_grouped(h1, Wqkv, ds, [L[t].up for t in QKV], qkv, alpha=ops.attn_q_scale(0.125), alpha_cols=D)
        else:
            ops.gemm_lora_grouped(h1, Wqkv, ds, [L[t].up for t in QKV], qkv)
        q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        if not FOLD_Q_SCALE:
            ops.scale_bf16_2d(q, ops.attn_q_scale(0.125), out=q)
        return q, k, v

    def _qkv_bwd(self, dqkv, Wqkv):
        """dh1 = [dq | dk | dv] . [Wq; Wk; Wv] + [vs_q | vs_k | vs_v] . [down_q; down_k; down_v] as ONE GEMM (the
        reference sums the three inputs' gradients in bf16; here one f32 sum, one rounding); the adapters'
        gradients per target as LoRALinearNF4.backward_adapters."""
        M, D, L = dqkv.shape[0], self.inner, self.lin
        r = L[QKV[0]].down.shape[0]
        vs = torch.empty(M, 3 * r, dtype=BF16, device=dqkv.device)
        ups = [L[t].up for t in QKV]
        grouped = _adjacent(ups) and len({L[t].scale for t in QKV}) == 1
        if grouped:  # vs_q | vs_k | vs_v = s * [dq | dk | dv] . blockdiag(up_q, up_k, up_v), one launch
            ops.lora_proj_grouped(dqkv, D, ups[0], ups[0].numel(), 3, False, vs, alpha=L[QKV[0]].scale)
        for g, t in enumerate(QKV):
            L[t].backward_adapters(dqkv[:, g * D:(g + 1) * D], vs_out=vs[:, g * r:(g + 1) * r], vs_ready=grouped)
        downs = [L[t].down for t in QKV]
        if _adjacent(downs):
            stacked = torch.as_strided(downs[0], (3 * r, D), (D, 1))  # the flat layout keeps them side by side
        else:
            stacked = torch.cat(downs, 0)  # standalone blocks: a copy of 3 x [r, dim]
        dh1 = torch.empty(M, D, dtype=BF16, device=dqkv.device)
        return ops.gemm_lora(dqkv, Wqkv, False, vs, stacked, M, D, 3 * D, dh1)

    def _attn_bwd(self, q, k, v, o, lse, do, B, n, nk, out=None):
        H = self.heads
        dq, dk, dv = out if out is not None else (torch.empty_like(q), torch.empty_like(k), torch.empty_like(v))
        delta = torch.empty_like(lse)
        ops.attn_bwd(ops._t4(q, B, n, H), ops._t4(k, B, nk, H), ops._t4(v, B, nk, H), ops._t4(o, B, n, H),
                     ops._t4(do, B, n, H), lse, delta, None, ops._t4(dq, B, n, H), ops._t4(dk, B, nk, H),
                     ops._t4(dv, B, nk, H), B, H, n, n, nk, nk=nk)
        return dq, dk, dv

    def forward(self, x: torch.Tensor, ctx: torch.Tensor, B: int, n: int, nc: int, save: bool = True) -> torch.Tensor:
        """x [B*n, dim] bf16, ctx [B*nc, context_dim] bf16 -> [B*n, dim] bf16 (denoiser.py:258-280)."""
        L = self.lin
        kv = self.ctx_kv
        self.ctx_kv = None
        if kv is not None and kv[2] != _ctx_key(ctx):
            kv = None  # projected for another context (or a stale precompute): project this one here
        kv = kv[:2] if kv is not None else None
        # the block's bases, one launch (the cross-attention k / v ones only when not projected already)
        Wb = dequant_bases(L, TARGETS if kv is None else [t for t in TARGETS if t not in ("attn2.to_k", "attn2.to_v")],
                           self.device)
        if self._fuse_qkv(Wb):
            h1, m1, r1, ds1 = self._ln_lora(x, "norm1", QKV)
            q, k, v = self._qkv_fwd(h1, Wb["attn1.qkv"], save, ds=ds1)
        else:
            h1, m1, r1 = ops.layernorm_fwd(x, *self.norm["norm1"])
            q, k, v = (L[f"attn1.to_{c}"].forward(h1, save, W=Wb.get(f"attn1.to_{c}"),
                                                  out_scale=self._q_out_scale() if c == "q" else 1.0) for c in "qkv")
            q = q if FOLD_Q_SCALE else self._qs(q)
        o1, lse1 = self._attn_fwd(q, k, v, B, n, n)
        x1 = L["attn1.to_out.0"].forward(o1, save, resid=x, W=Wb.get("attn1.to_out.0"))
        h2, m2, r2, ds2 = self._ln_lora(x1, "norm2", ["attn2.to_q"])
        q2 = L["attn2.to_q"].forward(h2, save, W=Wb.get("attn2.to_q"), ds=ds2, out_scale=self._q_out_scale())
        q2 = q2 if FOLD_Q_SCALE else self._qs(q2)
        if kv is not None:
            k2, v2 = kv
        else:
            k2 = L["attn2.to_k"].forward(ctx, save, W=Wb.get("attn2.to_k"))
            v2 = L["attn2.to_v"].forward(ctx, save, W=Wb.get("attn2.to_v"))
        o2, lse2 = self._attn_fwd(q2, k2, v2, B, n, nc)
        x2 = L["attn2.to_out.0"].forward(o2, save, resid=x1, W=Wb.get("attn2.to_out.0"))
        h3, m3, r3, ds3 = self._ln_lora(x2, "norm3", ["ff.net.0.proj"])
        x12 = L["ff.net.0.proj"].forward(h3, save, W=Wb.get("ff.net.0.proj"), ds=ds3)
        f2 = L["ff.net.2"]
        ds_f2 = None
        if FUSED_GEGLU_LORA_FWD and f2.skinny and x12.shape[1] % 256 == 0:
            ds_f2 = torch.empty(x12.shape[0], 16, dtype=BF16, device=self.device)
            gg = ops.geglu_fwd_lora(x12, f2.down, f2.scale, ds_f2)
        else:
            gg = ops.geglu_fwd(x12)
        y = f2.forward(gg, save, resid=x2, W=Wb.get("ff.net.2"), ds=ds_f2)
        self._st = dict(B=B, n=n, nc=nc, x=x, x1=x1, x2=x2, m=(m1, m2, m3), r=(r1, r2, r3), q=q, k=k, v=v, o1=o1,
                        lse1=lse1, q2=q2, k2=k2, v2=v2, o2=o2, lse2=lse2, x12=x12) if save else None
        return y

    def backward(self, dy: torch.Tensor, need_dctx: bool = True, vs: torch.Tensor | None = None,
                 prev_ff2: "LoRALinearNF4 | None" = None):
        """Returns (dx, dctx); accumulates every adapter's g_down / g_up (norms and NF4 bases frozen). The ten
        targets' adapter-gradient reduces run as one batched launch at the end (ops.lora_wgrad_batch).
        need_dctx=False: the context needs no gradient (the reference's text-encoder states are produced under
        no_grad, train/sdxl/flow_match.py:115-124), so the to_k / to_v input-gradient GEMMs are skipped.
        vs: ff.net.2's input-gradient LoRA operand s * dy . up, already computed by the caller (the next block's
        norm1 backward). prev_ff2: the ff.net.2 of the block before this one, which consumes dx as its output
        gradient -- its vs is then emitted by this block's norm1 backward (ops.layernorm_bwd_lora) into
        self.vs_prev (None where the fused form does not apply)."""
        with ops.lora_wgrad_batch(side=lora_side(self.device)):
            return self._backward(dy, need_dctx, vs, prev_ff2)

    def _backward(self, dy: torch.Tensor, need_dctx: bool = True, vs_ff2=None, prev_ff2=None):
        st, L = self._st, self.lin
        B, n, nc = st["B"], st["n"], st["nc"]
        m1, m2, m3 = st["m"]
        r1, r2, r3 = st["r"]
        # the bases of the input-gradient GEMMs about to run, one launch (to_k / to_v of the context only when
        # the context needs a gradient)
        Wb = dequant_bases(L, [t for t in TARGETS if need_dctx or t not in ("attn2.to_k", "attn2.to_v")], self.device)
        dgg = L["ff.net.2"].backward(dy, W=Wb.get("ff.net.2"), vs=vs_ff2)
        f0 = L["ff.net.0.proj"]
        # fused: 49 vs 70 us for the pair at M = 4224, F = 5120; 108 vs 118 us at M = 16896, F = 2560 (r06gd)
        if FUSED_GEGLU_LORA and f0.skinny and st["x12"].shape[1] % 256 == 0:
            vs_f0 = torch.empty(dgg.shape[0], 16, dtype=BF16, device=self.device)
            dx12 = ops.geglu_bwd_lora(dgg, st["x12"], f0.up, f0.scale, vs_f0)
        else:
            vs_f0 = None
            dx12 = ops.geglu_bwd(dgg, st["x12"])
        dh3 = f0.backward(dx12, W=Wb.get("ff.net.0.proj"), vs=vs_f0)
        dx2, vs_o2 = self._ln_bwd_lora(dh3, st["x2"], m3, r3, "norm3", dy, "attn2.to_out.0")
        do2 = L["attn2.to_out.0"].backward(dx2, W=Wb.get("attn2.to_out.0"), vs=vs_o2)
        D = self.inner
        dkv2 = torch.empty(B * nc, 2 * D, dtype=BF16, device=self.device)  # [dk2 | dv2]: one grouped vs launch
        dq2, dk2, dv2 = self._attn_bwd(st["q2"], st["k2"], st["v2"], st["o2"], st["lse2"], do2, B, n, nc,
                                       out=(torch.empty_like(st["q2"]), dkv2[:, :D], dkv2[:, D:]))
        dh2 = L["attn2.to_q"].backward(dq2, W=Wb.get("attn2.to_q"))
        KVT = ("attn2.to_k", "attn2.to_v")
        vs_kv = None
        if all(L[t].skinny for t in KVT) and _adjacent([L[t].up for t in KVT]) and L[KVT[0]].scale == L[KVT[1]].scale:
            vs_kv = torch.empty(B * nc, 32, dtype=BF16, device=self.device)
            ops.lora_proj_grouped(dkv2, D, L[KVT[0]].up, L[KVT[0]].up.numel(), 2, False, vs_kv, alpha=L[KVT[0]].scale)
        dck = L["attn2.to_k"].backward(dk2, need_dctx, W=Wb.get("attn2.to_k"),
                                       vs=None if vs_kv is None else vs_kv[:, :16])
        dcv = L["attn2.to_v"].backward(dv2, need_dctx, W=Wb.get("attn2.to_v"),
                                       vs=None if vs_kv is None else vs_kv[:, 16:])
        dctx = ops.add_bf16(dck, dcv) if need_dctx else None
        dx1, vs_o1 = self._ln_bwd_lora(dh2, st["x1"], m2, r2, "norm2", dx2, "attn1.to_out.0")
        do1 = L["attn1.to_out.0"].backward(dx1, W=Wb.get("attn1.to_out.0"), vs=vs_o1)
        if self._fuse_qkv(Wb):
            dqkv = torch.empty(B * n, 3 * self.inner, dtype=BF16, device=self.device)
            D = self.inner
            self._attn_bwd(st["q"], st["k"], st["v"], st["o1"], st["lse1"], do1, B, n, n,
                           out=(dqkv[:, :D], dqkv[:, D:2 * D], dqkv[:, 2 * D:]))
            dh1 = self._qkv_bwd(dqkv, Wb["attn1.qkv"])
        else:
            dq, dk, dv = self._attn_bwd(st["q"], st["k"], st["v"], st["o1"], st["lse1"], do1, B, n, n)
            dh1 = ops.add_bf16(ops.add_bf16(L["attn1.to_q"].backward(dq, W=Wb.get("attn1.to_q")),
                                            L["attn1.to_k"].backward(dk, W=Wb.get("attn1.to_k"))),
                               L["attn1.to_v"].backward(dv, W=Wb.get("attn1.to_v")))
        self.vs_prev = None
        if prev_ff2 is not None and FUSED_LN_BWD_PREV:
            dx, self.vs_prev = self._ln_bwd_lora(dh1, st["x"], m1, r1, "norm1", dx1, prev_ff2)
        else:
            dx = ops.layernorm_bwd(dh1, st["x"], m1, r1, self.norm["norm1"][0], dres=dx1)
        return dx, dctx

    def lora_grads(self) -> dict[str, torch.Tensor]:
        out = {}
        for t, l in self.lin.items():
            out[f"{t}.lora_down.weight"] = l.g_down
            out[f"{t}.lora_up.weight"] = l.g_up
        return out


class NF4Linear:
    """A frozen NF4 Linear without adapters (SpatialTransformer proj_in / proj_out): vpt_gemm_nf4 both ways."""

    def __init__(self, base: NF4Weight, bias: torch.Tensor | None, base_mode: str | None = None):
        self.base, self.bias = base, bias
        self.base_mode = base_mode or DEFAULT_BASE_MODE
        if base.shape[0] % 64 or base.shape[1] % 64:
            raise NotImplementedError("NF4Linear: in / out features must be multiples of 64")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = torch.empty(x.shape[0], self.base.shape[0], dtype=BF16, device=x.device)
        if self.base_mode == "inline":
            return ops.gemm_nf4(x, self.base, True, y, bias=self.bias)
        return ops.linear(x, base_weight(self.base, self.base_mode, x.device), bias=self.bias, out=y)

    def backward(self, dy: torch.Tensor) -> torch.Tensor:
        dx = torch.empty(dy.shape[0], self.base.shape[1], dtype=BF16, device=dy.device)
        if self.base_mode == "inline":
            return ops.gemm_nf4(dy, self.base, False, dx)
        return ops.linear_dgrad(dy, base_weight(self.base, self.base_mode, dy.device), out=dx)


def _nf4_or_dense(wt, code2, device):
    if isinstance(wt, dict):
        return NF4Weight.from_state(wt, device)
    if code2 is None:
        raise ValueError("dense base weights need the dynamic map `code2` to quantise")
    return NF4Weight.quantize(wt.to(device), code2)


class SDXLSpatialTransformer:
    """SpatialTransformer.forward (src/models/sdxl/denoiser.py:283-365) on the HIP kernels, QLoRA-trained:
    GroupNorm(32, C, eps 1e-6) on the NCHW stage activation (vpt_groupnorm_fwd) -> NCHW->tokens
    (vpt_transpose_add) -> proj_in (NF4) -> `depth` SDXLTransformerBlocks (LoRA on their 10 Linears) ->
    proj_out (NF4) -> tokens->NCHW + residual (vpt_transpose_add with the add fused). The backward returns the
    input and context gradients and accumulates every adapter's gradient (GroupNorm / proj weights frozen).
    State-dict names are the reference's (`norm.*`, `proj_in.*`, `transformer_blocks.{i}.<target>.linear.*`,
    `.lora_down.weight`, `.lora_up.weight`, `norm{1,2,3}.*`, `proj_out.*`)."""

    def __init__(self, C: int, heads: int, depth: int, context_dim: int, rank: int, alpha: float, sd: dict,
                 code2=None, device="cuda", groups: int = 32):
        self.C, self.heads, self.depth, self.groups = C, heads, depth, groups
        self.inner = heads * 64
        self.device = device
        self.norm_w = sd["norm.weight"].to(device, BF16).contiguous()
        self.norm_b = sd["norm.bias"].to(device, BF16).contiguous()
        self.proj_in = NF4Linear(_nf4_or_dense(sd["proj_in.weight"], code2, device),
                                 sd["proj_in.bias"].to(device, BF16).contiguous())
        self.proj_out = NF4Linear(_nf4_or_dense(sd["proj_out.weight"], code2, device),
                                  sd["proj_out.bias"].to(device, BF16).contiguous())
        self.blocks = []
        for i in range(depth):
            pre = f"transformer_blocks.{i}."
            self.blocks.append(SDXLTransformerBlock(self.inner, heads, context_dim, rank, alpha,
                                                    {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)},
                                                    code2=code2, device=device))
        self._st = None

    def forward(self, x: torch.Tensor, ctx: torch.Tensor, B: int, HW: int, nc: int, save: bool = True) -> torch.Tensor:
        """x NCHW bf16 [B, C, HW] (contiguous), ctx [B*nc, context_dim] -> NCHW bf16 [B, C, HW]."""
        C, G = self.C, self.groups
        h, mean, rstd = ops.groupnorm_fwd(x, self.norm_w, self.norm_b, B, C, G, HW)
        tok = ops.transpose_add(h, B, C, HW)                                  # [B, HW, C]
        t = self.proj_in.forward(tok.view(B * HW, C))
        for blk in self.blocks:
            t = blk.forward(t, ctx, B, HW, nc, save)
        u = self.proj_out.forward(t)
        y = ops.transpose_add(u.view(B, HW, C), B, HW, C, add=x)              # [B, C, HW] + residual
        self._st = dict(B=B, HW=HW, x=x, mean=mean, rstd=rstd) if save else None
        return y

    def backward(self, dy: torch.Tensor, need_dctx: bool = True):
        """dy NCHW [B, C, HW] -> (dx NCHW, dctx [B*nc, context_dim] or None with need_dctx=False)."""
        st = self._st
        B, HW, C, G = st["B"], st["HW"], self.C, self.groups
        du = ops.transpose_add(dy, B, C, HW)                                  # tokens [B, HW, C]
        dt = self.proj_out.backward(du.view(B * HW, C))
        dctx = None
        vs = None  # ff.net.2's vs of the block below, emitted by the norm1 backward of the block above
        for i in reversed(range(len(self.blocks))):
            blk = self.blocks[i]
            dt, dc = blk.backward(dt, need_dctx, vs=vs, prev_ff2=self.blocks[i - 1].lin["ff.net.2"] if i else None)
            vs = blk.vs_prev
            if need_dctx:
                dctx = dc if dctx is None else ops.add_bf16(dctx, dc)
        dtok = self.proj_in.backward(dt)
        dh = ops.transpose_add(dtok.view(B, HW, C), B, HW, C)                 # NCHW
        dx = ops.groupnorm_bwd(dh, st["x"], st["mean"], st["rstd"], self.norm_w, B, C, G, HW, dres=dy)
        return dx, dctx

    def lora_grads(self) -> dict[str, torch.Tensor]:
        out = {}
        for i, blk in enumerate(self.blocks):
            for k, v in blk.lora_grads().items():
                out[f"transformer_blocks.{i}.{k}"] = v
        return out
