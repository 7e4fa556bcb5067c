"""JiT denoiser forward/backward executor on the HIP kernels (no autograd in the hot path).

Restates JiT.forward (src/models/jit/denoiser.py:969-1124) and its backward as an explicit
schedule of libvpt_hip.so launches over pre-allocated HBM buffers:

  token layout  x[b][row][D], rows = N_p + 6 + T + n_ctx, order patches | image-size | time | ctx
                (the reference concatenates/strips context per block; here the context rows are
                always present and simply re-filled before every context block, and masked out as
                keys — n = N_p + 6 + T — in the blocks before context_start_block).
  per block     RMSNorm -> QKV GEMM (+bias) -> QK-RMSNorm+RoPE -> flash attention (key-padding
                bias, no [B,H,N,N] mask) -> O GEMM (+bias +residual) -> RMSNorm -> W1|W2 GEMM
                (+bias) -> SwiGLU -> W3 GEMM (+bias +residual)
  backward      mirrors it; weight grads are f32 (split-K wgrad GEMMs, deterministic slab reduce),
                bias/norm grads are deterministic two-stage reductions.

Activations saved for backward are kept (no recompute): ~28 KB/token/block at D=768, i.e.
~11 GB for JiT-B/16 at B=8 x 1024^2 — memory is laid out for 288 GB of HBM per GPU.
"""

from __future__ import annotations

import contextlib
import math

import torch

from . import ops
from .config import DenoiserConfig, check_supported
from .params import ParamLayout
from .rope import RopeCache

BF16, F32 = torch.bfloat16, torch.float32
NEG_INF = float("-inf")

# Module attributes (no environment switches; tools/c3_knob_ab.py assigns them in-process for same-box A/B runs),
# defaults = the measured faster form:
# QK-RMSNorm + RoPE forward inside the q|k|v GEMM's epilogue (vpt_linear_qknorm_rope) vs its own pass after it:
# +0.29 % per C3 step (r04e, same-box in-process A/B)
FUSED_QKNORM_FWD = True
# QK-RMSNorm + RoPE backward inside the attention backward's dQ / dK stores (vpt_attn_bwd_qknorm) vs its own pass:
# measured 0.76 % SLOWER per C3 step (r04e: the per-workgroup tail -- raw-row loads, RoPE tables, the LDS reduction of
# the weight-gradient partials -- costs more than the standalone memory-bound pass), so off
FUSED_QKNORM_BWD = False
# attention forward with the QK-norm score bound as a fixed softmax reference point (vpt_attn_fwd_qknorm): +0.2 %
FIXREF_ATTN_FWD = True
# The backward's weight-gradient GEMMs on a second HIP stream (the input-gradient chain stays on the caller's stream):
# nothing in the chain reads a weight gradient, so each wgrad runs beside the chain's next kernels and fills the CUs
# their last, partial round of work items leaves idle. Stream-ordered hand-offs only (events; no host sync).
CONCURRENT_WGRAD = True
# A/B knobs of the side stream: its HIP priority (0 = the default streams' level, -1 = high: level, r05x) and a factor on
# the wgrads' split-K count (ops.wgrad_splits sizes it to fill the chip alone)
WGRAD_STREAM_PRIORITY = 0
WGRAD_SPLIT_DIV = 1  # 2: C3 step -5.5 % (r05x) -- the wgrads then lag the chain's hand-off waits
WGRAD_SPLIT_MUL = 1
# The transformer blocks as MICRO_SPLIT independent sub-batches (B / MICRO_SPLIT sequences each) on their own streams,
# forward and input-gradient chain: every op there is row- or sequence-local, so the sub-batches need no exchange (the
# forward is bitwise the one-batch forward; the backward's weight gradients still cover the whole batch); one
# sub-batch's kernels fill the CUs the other's leave idle in their last, partial round of work items (the GEMMs' wave
# quantisation, the attention grids' tails). 2: C3 step +1.8 % (r05za), +2.5 % with checkpointing (r05zi). Lanes are
# used only when each keeps at least MICRO_SPLIT_MIN_ROWS token rows: at C2 (512^2, B=16: 8.7k rows per lane) lanes in
# forward AND backward were -3.6 % (r05zo, threshold 12288 then), forward-only lanes are +2.3 % (r05zzc), so the
# threshold now admits C2 and keeps small batches (C1: 0.6k rows per lane) on one stream. 1 = one stream. Needs
# B % MICRO_SPLIT == 0.
MICRO_SPLIT = 2
MICRO_SPLIT_MIN_ROWS = 8192
# Where the lanes run (r05zr, same-box A/Bs at C3 with the other half on): in the forward +2.5 %; in the backward's
# input-gradient chain -1.2 % (there the side-stream weight gradients already fill the chain's partial rounds, and the
# lanes' extra hand-offs cost more than they fill), so the backward runs one lane by default.
MICRO_SPLIT_FWD = True
MICRO_SPLIT_BWD = False
# The attention backward on the persistent work-queue kernel (vpt_attn_bwd_q: resident blocks pulling dK/dV and dQ items
# from per-XCD queues, the next item's first tile staged under the current item's last; bitwise the one-launch grid).
# Measured slower (tools/attn_queue_ab.py, r06b / r06c, same box, interleaved): C3 1.371 vs 1.348 ms (+1.7 %), C2 0.267 vs
# 0.232 ms (+15 %) with the ticket pulled in the item's prologue; +3.9 % / +20 % with it taken one item ahead (its return
# then waited at the first tile's vmcnt(0)); C3 step -0.54 % (r06b). Each item still pays a vmcnt(0) on the previous
# item's epilogue stores (vector-memory counters retire in issue order) and the atomic's round trip, which the
# dispatcher's block launch does not. Off.
ATTN_BWD_QUEUE = False
# Gradient checkpointing's per-block recompute in the backward as forward lanes too (while the backward itself runs one
# lane); A/B knob
MICRO_SPLIT_RECOMPUTE = True


def _lanes(B: int, rows: int, device) -> int:
    """The number of sub-batch lanes for a batch of B sequences of `rows` token rows."""
    S = MICRO_SPLIT
    if S > 1 and B % S == 0 and (B // S) * rows >= MICRO_SPLIT_MIN_ROWS and torch.device(device).type == "cuda":
        return S
    return 1


class _SubPool:
    """Row slice h of n of every buffer a _Pool hands out (first dimension = the sub-batch's share)."""

    def __init__(self, pool, h: int, n: int):
        self.pool, self.h, self.n = pool, h, n

    def get(self, name: str, shape, dtype=BF16, zero: bool = False) -> torch.Tensor:
        # the pooled buffer is shared by every lane: only this lane's slice may be zeroed, on this lane's stream
        full = self.pool.get(name, (shape[0] * self.n,) + tuple(shape[1:]), dtype)
        v = full[self.h * shape[0]:(self.h + 1) * shape[0]]
        if zero:
            v.zero_()
        return v


class _Pool:
    """Named, growable device buffers (views into cached storages).

    A storage is allocated (zero-filled: rows a kernel never writes, e.g. a pre-context block's context rows, must stay
    finite) on the first use of a name or when a larger bucket needs it to grow. That may happen on any of the engine's
    streams (sub-batch lanes, the weight-gradient stream), and the view it returns may then be handed to kernels on any
    other of them (a buffer got on the step's stream is written by the lanes), so an allocation is made safe for all of
    them without a host sync:
    - the zero fill runs on the allocating stream, and every other engine stream waits (stream-ordered) for an event
      recorded after it before anything enqueued on it later -- no kernel on any stream can touch the new storage
      before its fill is complete;
    - a replaced storage is marked used by every engine stream (record_stream), so the caching allocator does not hand
      its memory out again before the work those streams have enqueued so far is done."""

    def __init__(self, device, streams=None):
        self.device = device
        self.store: dict[str, torch.Tensor] = {}
        self._streams = streams  # callable -> the engine's streams

    def get(self, name: str, shape, dtype=BF16, zero: bool = False) -> torch.Tensor:
        n = 1
        for s in shape:
            n *= s
        cur = self.store.get(name)
        if cur is None or cur.numel() < n or cur.dtype != dtype:
            cuda = self.device.type == "cuda"
            if cur is not None and cuda:
                for st in self._engine_streams():
                    cur.record_stream(st)
            cur = torch.zeros(max(n, 1), dtype=dtype, device=self.device)
            if cuda:
                here = torch.cuda.current_stream(self.device)
                ev = torch.cuda.Event()
                ev.record(here)
                for st in self._engine_streams():
                    if st != here:
                        st.wait_event(ev)
            self.store[name] = cur
        v = cur[:n].view(*shape)
        if zero:
            v.zero_()
        return v

    def _engine_streams(self):
        out = [torch.cuda.current_stream(self.device), torch.cuda.default_stream(self.device)]
        if self._streams is not None:
            out += [s for s in self._streams() if s is not None]
        return out


class JiTEngine:
    def __init__(self, cfg: DenoiserConfig, device="cuda", n_classes: int | None = None,
                 params: torch.Tensor | None = None, grads: torch.Tensor | None = None):
        check_supported(cfg)
        self.cfg = cfg
        self.device = torch.device(device)
        self.n_classes = n_classes
        self.layout = ParamLayout(cfg, n_classes)
        self.params = params if params is not None else torch.zeros(self.layout.total, dtype=BF16, device=self.device)
        self.grads = grads if grads is not None else torch.zeros(self.layout.total, dtype=F32, device=self.device)
        self.pool = _Pool(self.device, self._pool_streams)
        self.pool_infer = _Pool(self.device, self._pool_streams)  # no-grad forwards never clobber saved activations
        self.rope = RopeCache(cfg, self.device)
        self.D = cfg.hidden_size
        self.F = cfg.mlp_hidden_padded  # zero-padded SwiGLU width (vpt.params.ParamSpec)
        self.H = cfg.num_heads
        self.T = cfg.num_time_tokens
        self._state = None
        self.gradient_checkpointing = False
        self._wstream = None  # the weight-gradient stream (CONCURRENT_WGRAD), created on first use
        self._mstreams = []   # the sub-batch streams (MICRO_SPLIT)
        self._bind()

    def _pool_streams(self):
        return list(self._mstreams) + ([self._wstream] if self._wstream is not None else [])

    # ------------------------------------------------------------------ parameter views
    def _bind(self):
        L, P, G = self.layout, self.params, self.grads
        D, F = self.D, self.F
        self.p = {s.name: L.view(P, s.name) for s in L.specs}
        self.g = {s.name: L.view(G, s.name) for s in L.specs}
        self.blk = []
        for i in range(self.cfg.depth):
            pre = f"blocks.{i}."
            d = {}
            for store, src in (("p", P), ("g", G)):
                d[store + "wqkv"] = L.span(src, pre + "attn.to_q.weight", pre + "attn.to_v.weight", (3 * D, D))
                d[store + "bqkv"] = L.span(src, pre + "attn.to_q.bias", pre + "attn.to_v.bias", (3 * D,))
                d[store + "wo"] = L.view(src, pre + "attn.to_o.weight")
                d[store + "bo"] = L.view(src, pre + "attn.to_o.bias")
                d[store + "qk_norm"] = L.span(src, pre + "attn.q_norm.weight", pre + "attn.k_norm.weight", (128,))
                d[store + "n1"] = L.view(src, pre + "norm1.weight")
                d[store + "n2"] = L.view(src, pre + "norm2.weight")
                d[store + "w12"] = L.span(src, pre + "mlp.w_1.weight", pre + "mlp.w_2.weight", (2 * F, D))
                d[store + "b12"] = L.span(src, pre + "mlp.w_1.bias", pre + "mlp.w_2.bias", (2 * F,))
                d[store + "w3"] = L.phys(src, pre + "mlp.w_3.weight")
                d[store + "b3"] = L.view(src, pre + "mlp.w_3.bias")
            self.blk.append(d)
        fin = {}
        for store, src in (("p", P), ("g", G)):
            fin[store + "n"] = L.view(src, "final_layer.norm_final.weight")
            fin[store + "w12"] = L.span(src, "final_layer.mlp.w_1.weight", "final_layer.mlp.w_2.weight", (2 * F, D))
            fin[store + "b12"] = L.span(src, "final_layer.mlp.w_1.bias", "final_layer.mlp.w_2.bias", (2 * F,))
            fin[store + "w3"] = L.phys(src, "final_layer.mlp.w_3.weight")
            fin[store + "b3"] = L.view(src, "final_layer.mlp.w_3.bias")
            fin[store + "wl"] = L.view(src, "final_layer.linear.weight")
            fin[store + "bl"] = L.view(src, "final_layer.linear.bias")
        self.fin = fin

    # ------------------------------------------------------------------ weights
    def init_weights(self, seed: int = 0):
        """JiT.initialize_weights (denoiser.py:764-798) + ClassEncoder.initialize_weights
        (class_encoder.py:124-125): Linear/patch conv/time_position_embeds N(0, 0.02), biases 0,
        RMSNorm weights 1, class embedding N(0, 0.02) (padding row included)."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        for s in self.layout.specs:
            n = s.name
            if n.endswith(("norm1.weight", "norm2.weight", "q_norm.weight", "k_norm.weight", "norm_final.weight")):
                v = torch.ones(s.shape)
            elif n.endswith(".bias"):
                v = torch.zeros(s.shape)
            else:
                v = torch.randn(s.shape, generator=g) * 0.02
            self.p[n].copy_(v.to(BF16))

    def load_state_dict(self, sd: dict[str, torch.Tensor], strict: bool = True):
        missing = [n for n in self.p if n not in sd]
        unexpected = [k for k in sd if k not in self.p]
        if strict and (missing or unexpected):
            raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
        for n, t in sd.items():
            if n in self.p:
                if tuple(t.shape) != tuple(self.p[n].shape):
                    raise ValueError(f"{n}: shape {tuple(t.shape)} != {tuple(self.p[n].shape)}")
                self.p[n].copy_(t.to(device=self.device, dtype=BF16))

    def state_dict(self) -> dict[str, torch.Tensor]:
        return {n: v.detach().clone() for n, v in self.p.items()}

    # ------------------------------------------------------------------ shapes
    def shape_info(self, B: int, H: int, W: int, n_ctx: int):
        P = self.cfg.patch_size
        if H % P or W % P:
            raise ValueError(f"image {H}x{W} is not a multiple of patch {P}")
        hp, wp = H // P, W // P
        np_ = hp * wp
        rows = np_ + 6 + self.T + n_ctx
        return hp, wp, np_, rows

    # ------------------------------------------------------------------ forward
    def forward(self, zp: torch.Tensor, B: int, H: int, W: int, t_vals: torch.Tensor, size_vals: torch.Tensor,
                ctx_raw: torch.Tensor, kbias: torch.Tensor | None, n_ctx: int, save: bool = True) -> torch.Tensor:
        """zp [B*N_p, C*P*P] bf16 patchified input (im2col order c,ky,kx); t_vals [B] f32 (the
        bf16-rounded timestep times timestep_scale); size_vals [6B] f32; ctx_raw [B*n_ctx,
        context_dim] bf16; kbias [B, rows] f32 additive key bias (0 / -inf) or None.
        Returns the final-layer output in patch layout [B*N_p, P*P*C] (per patch (py, px, c))."""
        cfg, D, F, Hh = self.cfg, self.D, self.F, self.H
        pool = self.pool if save else self.pool_infer
        hp, wp, np_, rows = self.shape_info(B, H, W, n_ctx)
        M = B * rows
        n_pre = np_ + 6 + self.T           # tokens attended before context_start_block
        cos_t, sin_t = self.rope.get(hp, wp, n_ctx)
        p = self.p
        # --- embeddings (denoiser.py:982-1009)
        temb_in = ops.timestep_embed(t_vals, pool.get("temb_in", (B, 256)))
        t_a1 = ops.linear(temb_in, p["time_embedder.mlp.0.weight"], p["time_embedder.mlp.0.bias"], out=pool.get("t_a1", (B, D)))
        t_h1 = ops.silu(t_a1, pool.get("t_h1", (B, D)))
        temb = ops.linear(t_h1, p["time_embedder.mlp.2.weight"], p["time_embedder.mlp.2.bias"], out=pool.get("temb", (B, D)))
        semb_in = ops.timestep_embed(size_vals, pool.get("semb_in", (6 * B, 256)))
        s_a1 = ops.linear(semb_in, p["image_size_embedder.mlp.0.weight"], p["image_size_embedder.mlp.0.bias"],
                          out=pool.get("s_a1", (6 * B, D)))
        s_h1 = ops.silu(s_a1, pool.get("s_h1", (6 * B, D)))
        semb = ops.linear(s_h1, p["image_size_embedder.mlp.2.weight"], p["image_size_embedder.mlp.2.bias"],
                          out=pool.get("semb", (6 * B, D)))
        ctx = None
        if n_ctx:
            ctx = ops.linear(ctx_raw, p["context_embedder.weight"], p["context_embedder.bias"], out=pool.get("ctx", (B * n_ctx, D)))
        bd = cfg.bottleneck_dim
        w1 = p["patch_embedder.proj_1.weight"].view(bd, -1)
        w2 = p["patch_embedder.proj_2.weight"].view(D, bd)
        pe1 = ops.linear(zp, w1, out=pool.get("pe1", (B * np_, bd)))
        pe2 = ops.linear(pe1, w2, p["patch_embedder.proj_2.bias"], out=pool.get("pe2", (B * np_, D)))
        x = pool.get("x0", (M, D))
        ops.assemble_tokens(pe2, semb, temb, p["time_position_embeds"], ctx, n_ctx, B, np_, rows, x)
        # --- blocks (denoiser.py:1087-1113)
        S = _lanes(B, rows, self.device) if MICRO_SPLIT_FWD else 1
        if S > 1:
            main = torch.cuda.current_stream(self.device)
            while len(self._mstreams) < S:
                self._mstreams.append(torch.cuda.Stream(device=self.device))
            subs = self._mstreams[:S]
            for st in subs:
                st.wait_stream(main)  # embeddings / assembled tokens written
            Bh, Mh = B // S, (B // S) * rows
            spools = [_SubPool(pool, h, S) for h in range(S)]
        for i, w in enumerate(self.blk):
            x_next = pool.get(f"x{i + 1}" if save else ("xa" if i % 2 == 0 else "xb"), (M, D))
            # gradient checkpointing (denoiser.py:945-967): only the block inputs x{i} are kept; the block's
            # intermediates go to one scratch set and are recomputed in backward
            tag = ("ck." if self.gradient_checkpointing else f"b{i}.") if save else "s."
            if S == 1:
                if n_ctx and self._ctx_refresh(i):
                    ops.ctx_rows(x, B, n_pre, rows, n_ctx, ctx=ctx)
                self._block_forward(i, x, x_next, tag, pool, B, rows, n_ctx, n_pre, kbias, cos_t, sin_t)
            else:
                for h in range(S):
                    with torch.cuda.stream(subs[h]):
                        xh, r0 = x[h * Mh:(h + 1) * Mh], h * Bh
                        if n_ctx and self._ctx_refresh(i):
                            ops.ctx_rows(xh, Bh, n_pre, rows, n_ctx, ctx=ctx[r0 * n_ctx:(r0 + Bh) * n_ctx])
                        self._block_forward(i, xh, x_next[h * Mh:(h + 1) * Mh], tag, spools[h], Bh, rows, n_ctx,
                                            n_pre, None if kbias is None else kbias[r0:r0 + Bh], cos_t, sin_t)
            x = x_next
        if S > 1:
            for st in subs:
                main.wait_stream(st)
        # --- final layer + (per-patch) output (denoiser.py:1115-1116, 535-543)
        f = self.fin
        M2 = B * np_
        xf = ops.copy_rows(x, rows, 0, np_, pool.get("xf", (M2, D)), B)
        xnf, rstdf = ops.rmsnorm_fwd(xf, f["pn"], pool.get("xnf", (M2, D)), pool.get("rstdf", (M2,), F32))
        f12, fh = ops.linear_swiglu(xnf, f["pw12"], f["pb12"], pool.get("f12", (M2, 2 * F)), pool.get("fh", (M2, F)))
        f3 = ops.linear(fh, f["pw3"], f["pb3"], out=pool.get("f3", (M2, D)))
        out = ops.linear(f3, f["pwl"], f["pbl"], out=pool.get("out", (M2, f["pwl"].shape[0])))
        self._state = dict(B=B, H=H, W=W, np_=np_, rows=rows, n_ctx=n_ctx, n_pre=n_pre, M=M, kbias=kbias,
                           zp=zp, ctx_raw=ctx_raw, cos=cos_t, sin=sin_t,
                           ckpt=self.gradient_checkpointing) if save else None
        return out

    def _block_forward(self, i, x, x_next, tag, pool, B, rows, n_ctx, n_pre, kbias, cos_t, sin_t):
        """JiTBlock.forward (denoiser.py:582-649) of block i: x -> x_next, intermediates under `tag`."""
        cfg, D, F, Hh = self.cfg, self.D, self.F, self.H
        w = self.blk[i]
        M = x.shape[0]
        n_i = rows if (n_ctx and self._ctx_present(i)) else n_pre
        xn1, rstd1 = ops.rmsnorm_fwd(x, w["pn1"], pool.get(tag + "xn1", (M, D)), pool.get(tag + "rstd1", (M,), F32))
        qs = ops.attn_q_scale(1.0 / math.sqrt(cfg.head_dim))  # q leaves pre-scaled for the attention kernels
        qkv_buf, qk_buf = pool.get(tag + "qkv", (M, 3 * D)), pool.get(tag + "qk", (M, 2 * D))
        wq, wk = w["pqk_norm"][:64], w["pqk_norm"][64:]
        if FUSED_QKNORM_FWD:  # q|k|v projection with the per-head QK-RMSNorm + RoPE in its epilogue
            qkv, qk = ops.linear_qknorm_rope(xn1, w["pwqkv"], w["pbqkv"], qkv_buf, qk_buf, wq, wk, cos_t, sin_t, rows,
                                             q_scale=qs)
        else:
            qkv = ops.linear(xn1, w["pwqkv"], w["pbqkv"], out=qkv_buf)
            qk = ops.qknorm_rope_fwd(qkv, wq, wk, cos_t, sin_t, rows, out=qk_buf, q_scale=qs)
        o = pool.get(tag + "o", (M, D))
        lse = pool.get(tag + "lse", (B, Hh, rows), F32)
        a4 = (ops._t4(qk, B, rows, Hh, 0), ops._t4(qk, B, rows, Hh, D), ops._t4(qkv, B, rows, Hh, 2 * D),
              ops._t4(o, B, rows, Hh, 0))
        if FIXREF_ATTN_FWD:
            ops.attn_fwd_qknorm(*a4, lse, kbias, wq, wk, B, Hh, rows, n_i, n_pre, 1.0 / math.sqrt(cfg.head_dim))
        else:
            ops.attn_fwd(*a4, lse, kbias, B, Hh, rows, n_i, n_pre, 1.0 / math.sqrt(cfg.head_dim))
        xm = ops.linear(o, w["pwo"], w["pbo"], resid=x, out=pool.get(tag + "xm", (M, D)))
        xn2, rstd2 = ops.rmsnorm_fwd(xm, w["pn2"], pool.get(tag + "xn2", (M, D)), pool.get(tag + "rstd2", (M,), F32))
        x12, h = ops.linear_swiglu(xn2, w["pw12"], w["pb12"], pool.get(tag + "x12", (M, 2 * F)),
                                   pool.get(tag + "h", (M, F)))
        ops.linear(h, w["pw3"], w["pb3"], resid=xm, out=x_next)

    def set_gradient_checkpointing(self, enable: bool = True):
        """JiT.set_gradient_checkpointing (denoiser.py:800-801): keep only block inputs, recompute in backward."""
        self.gradient_checkpointing = bool(enable)

    def _ctx_present(self, i: int) -> bool:
        cs = self.cfg.context_start_block
        return i >= cs

    def _ctx_refresh(self, i: int) -> bool:
        cs = self.cfg.context_start_block
        return i == cs or (not self.cfg.do_context_fuse and i > cs)

    # ------------------------------------------------------------------ backward
    def backward(self, dout: torch.Tensor, zero_grads: bool = True, on_ready=None,
                 overwritten: tuple = ()) -> torch.Tensor | None:
        """dout [B*N_p, P*P*C] bf16 gradient of the patch-layout output. Fills self.grads (f32;
        accumulates when zero_grads=False) and returns d(ctx_raw) [B*n_ctx, context_dim] bf16. `overwritten`: gradient
        names the caller writes with overwrite semantics after this backward (not zeroed here)."""
        st = self._state
        if st is None:
            raise RuntimeError("backward() needs a forward(save=True) first")
        cfg, pool, D, F, Hh = self.cfg, self.pool, self.D, self.F, self.H
        B, np_, rows, n_ctx, n_pre, M = st["B"], st["np_"], st["rows"], st["n_ctx"], st["n_pre"], st["M"]
        M2 = B * np_
        cos_t, sin_t = st["cos"], st["sin"]
        if zero_grads:
            # every gradient slice below is written with overwrite semantics when acc is False; only the slices this
            # backward does not write (the class-embedding table the trainer scatter-adds into, the context embedder
            # of a context-free batch) are zeroed, instead of a fill over the whole flat buffer
            self._zero_unwritten_grads(n_ctx, overwritten)
        acc = not zero_grads
        ws = pool.get("wgrad_ws", (self._ws_elems(max(M, M2)),), F32)
        f, g = self.fin, self.g
        # Weight gradients on the side stream: each waits (event) for its inputs on the main stream; the main stream
        # waits for a wgrad's event before it overwrites a buffer that wgrad reads (the ping-pong gradient buffers, the
        # partial-row buffers its reduce sums, the recomputed activations under checkpointing) -- see `settle`. The
        # workspace `ws` is used by the side stream alone, whose launches run in order.
        side = None
        if CONCURRENT_WGRAD and self.device.type == "cuda":
            if self._wstream is None or self._wstream.priority != WGRAD_STREAM_PRIORITY:
                self._wstream = torch.cuda.Stream(device=self.device, priority=WGRAD_STREAM_PRIORITY)
            side = self._wstream
        main = torch.cuda.current_stream(self.device) if side is not None else None
        on_side = side is not None
        self._wait_inputs = None

        def wgrad(dy, xin, out, bias=None, rows_sum=None):
            """weight gradient, and with `bias` the bias gradient in the same GEMM (vpt_linear_wgrad); rows_sum = an
            RMSNorm / QK-norm weight gradient's partial-row sum riding its reduce launch (vpt_linear_wgrad_rr).
            Returns the side stream's event after it (None without the side stream)."""
            Mr, N = dy.shape
            K = xin.shape[1]
            s = max(1, ops.wgrad_splits(N, K, Mr) * WGRAD_SPLIT_MUL // WGRAD_SPLIT_DIV)
            while s > 1 and Mr // s < 256:
                s -= 1
            while s > 1 and ops.linear_wgrad_workspace_bytes(Mr, N, K, s) > ws.numel() * 4:
                s -= 1

            def run():
                ops.linear_wgrad(dy, xin, out.view(N, K), accumulate=acc, splits=s, workspace=ws,
                                 bias_out=None if bias is None else bias.view(-1), rows_sum=rows_sum)
            if side is None or not on_side:
                run()
                return None
            if self._wait_inputs is not None:
                self._wait_inputs()  # every sub-batch lane wrote dy, xin and the partial rows
            else:
                side.wait_stream(main)  # dy, xin and the partial rows are written
            with torch.cuda.stream(side):
                run()
            ev = torch.cuda.Event()
            ev.record(side)
            return ev

        def settle(ev):
            """The main stream waits for the side stream up to `ev` (a wgrad's event; None = nothing pending)."""
            if ev is not None:
                main.wait_event(ev)

        # --- final layer
        f3, fh, f12, xnf, xf = (pool.get(n, s) for n, s in (("f3", (M2, D)), ("fh", (M2, F)), ("f12", (M2, 2 * F)),
                                                          ("xnf", (M2, D)), ("xf", (M2, D))))
        rstdf = pool.get("rstdf", (M2,), F32)
        wgrad(dout, f3, f["gwl"], f["gbl"])
        df3 = ops.linear_dgrad(dout, f["pwl"], out=pool.get("d_a", (M2, D)))
        wgrad(df3, fh, f["gw3"], f["gb3"])
        df12 = ops.linear_dgrad_swiglu(df3, f["pw3"], f12, pool.get("d_x12", (M2, 2 * F)),
                                       workspace=pool.get("d_h", (M2, F)))
        ev = wgrad(df12, xnf, f["gw12"], f["gb12"])
        dxnf = ops.linear_dgrad(df12, f["pw12"], out=pool.get("d_b", (M2, D)))
        dxf, part = ops.rmsnorm_bwd(dxnf, xf, rstdf, f["pn"], dx=pool.get("d_c", (M2, D)),
                                    dw_part=pool.get("rms_part", (ops.rmsnorm_bwd_blocks(max(M, M2)), D), F32))
        ops.reduce_rows(part[:ops.rmsnorm_bwd_blocks(M2)], f["gn"], acc)
        settle(ev)  # the blocks below reuse d_x12 and the gradient buffers the final layer's wgrads read
        if on_ready is not None:
            on_ready("final")  # every final_layer.* gradient is enqueued
        dx = pool.get("dx_a", (M, D))
        ops.copy_rows(dx, rows, 0, np_, dxf, B, reverse=True, zero_rest=True)  # token / context rows: zero
        # --- blocks in reverse. With MICRO_SPLIT = S > 1 (and the side stream) the input-gradient chain runs as S
        # independent sub-batches on their own streams ("lanes"), like the forward; every weight gradient -- and
        # norm1's weight-gradient reduce -- covers the whole batch on the side stream once all lanes produced its
        # inputs. S = 1: one lane, the caller's stream.
        S = _lanes(B, rows, self.device) if (side is not None and not FUSED_QKNORM_BWD and MICRO_SPLIT_BWD) else 1
        if S > 1:
            while len(self._mstreams) < S:
                self._mstreams.append(torch.cuda.Stream(device=self.device))
            lanes = self._mstreams[:S]
            for ln in lanes:
                ln.wait_stream(main)  # the final layer's dx / copy_rows and settle(ev) above
        else:
            lanes = [main]
        Bh, Mh = B // S, M // S
        nb_h, nq_h = ops.rmsnorm_bwd_blocks(Mh), ops.qknorm_rope_blocks(Mh)
        spools = [_SubPool(pool, h, S) for h in range(S)] if S > 1 else [pool]

        def rs(t, h):  # sub-batch h's rows of an [M, ...] buffer
            return t if S == 1 else t[h * Mh:(h + 1) * Mh]

        def bs(t, h):  # sub-batch h's sequences of a [B, ...] buffer
            return t if (S == 1 or t is None) else t[h * Bh:(h + 1) * Bh]

        def on(h):
            return torch.cuda.stream(lanes[h]) if S > 1 else contextlib.nullcontext()

        if side is not None:
            def side_wait():
                for ln in lanes:
                    side.wait_stream(ln)
            wait_inputs = side_wait

            def settle(ev):  # noqa: F811  (every lane waits)
                if ev is not None:
                    for ln in lanes:
                        ln.wait_event(ev)
        else:
            wait_inputs = None
        self._wait_inputs = wait_inputs

        dctx = pool.get("dctx", (max(B * n_ctx, 1), D), F32)  # written by the first refresh block's ctx_rows
        dctx_set = False
        dqkv = pool.get("d_qkv", (M, 3 * D))
        delta = pool.get("delta", (B, Hh, rows), F32)
        n_dw = ops.attn_bwd_dw_rows(B, Hh, rows)
        qk_dw = pool.get("qk_dw_part", (n_dw, 128), F32)  # q_norm | k_norm weight-gradient partials
        part1 = pool.get("rms_part1", (S * nb_h, D), F32)  # norm1's weight-gradient partial rows (per lane: nb_h)
        part2 = pool.get("rms_part2", (S * nb_h, D), F32)  # norm2's
        qkp = pool.get("qk_part", (S * nq_h, 128), F32)
        pre_zeroed = False
        scale = 1.0 / math.sqrt(cfg.head_dim)
        ck = st.get("ckpt", False)
        kbias = st["kbias"]
        ev_qkv = None  # the previous block's last side-stream event (its q|k|v wgrad, or norm1's reduce)
        ready = None   # that block's name for on_ready, announced once its gradients are waited for

        def settle_qkv():
            nonlocal ev_qkv, ready
            settle(ev_qkv)
            if ready is not None and on_ready is not None:
                if S > 1:
                    main.wait_event(ev_qkv)  # the bucket's collective is enqueued on the caller's stream
                on_ready(ready)  # every gradient of that block is complete in the main stream's order
            ev_qkv = None
            ready = None

        def wg(dy, xin, out, bias=None, rows_sum=None):
            """wgrad over the whole batch; the side stream waits for every lane first."""
            return wgrad(dy, xin, out, bias, rows_sum)

        for i in reversed(range(cfg.depth)):
            w = self.blk[i]
            tag = "ck." if ck else f"b{i}."
            x_in = pool.get(f"x{i}" if i > 0 else "x0", (M, D))
            if ck:
                settle_qkv()  # the recompute below overwrites the ck.* activations the previous block's wgrads read
                # recompute the block's intermediates from its saved input (x{i+1} is left untouched)
                xo = pool.get("ck.xout", (M, D))
                Sr = _lanes(B, rows, self.device) if (S == 1 and MICRO_SPLIT_FWD and MICRO_SPLIT_RECOMPUTE) else 1
                if Sr > 1:  # the recompute as forward lanes (bitwise the one-lane recompute), joined on main
                    while len(self._mstreams) < Sr:
                        self._mstreams.append(torch.cuda.Stream(device=self.device))
                    subs, cur = self._mstreams[:Sr], torch.cuda.current_stream(self.device)
                    for st_r in subs:
                        st_r.wait_stream(cur)
                    Bhr, Mhr = B // Sr, M // Sr
                    for hh in range(Sr):
                        with torch.cuda.stream(subs[hh]):
                            self._block_forward(i, x_in[hh * Mhr:(hh + 1) * Mhr], xo[hh * Mhr:(hh + 1) * Mhr], tag,
                                                _SubPool(pool, hh, Sr), Bhr, rows, n_ctx, n_pre,
                                                None if kbias is None else kbias[hh * Bhr:(hh + 1) * Bhr], cos_t, sin_t)
                    for st_r in subs:
                        cur.wait_stream(st_r)
                else:
                    for hh in range(S):
                        with on(hh):
                            self._block_forward(i, rs(x_in, hh), rs(xo, hh), tag, spools[hh], Bh, rows, n_ctx, n_pre,
                                                bs(kbias, hh), cos_t, sin_t)
            xn1, qkv, qk, o = (pool.get(tag + n, s) for n, s in (("xn1", (M, D)), ("qkv", (M, 3 * D)),
                                                                 ("qk", (M, 2 * D)), ("o", (M, D))))
            xm, xn2, x12, h = (pool.get(tag + n, s) for n, s in (("xm", (M, D)), ("xn2", (M, D)),
                                                                 ("x12", (M, 2 * F)), ("h", (M, F))))
            rstd1, rstd2 = pool.get(tag + "rstd1", (M,), F32), pool.get(tag + "rstd2", (M,), F32)
            lse = pool.get(tag + "lse", (B, Hh, rows), F32)
            n_i = rows if (n_ctx and self._ctx_present(i)) else n_pre
            d_x12, d_h, d_b = pool.get("d_x12", (M, 2 * F)), pool.get("d_h", (M, F)), pool.get("d_b", (M, D))
            dx_b, d_o, dx_a = pool.get("dx_b", (M, D)), pool.get("d_o", (M, D)), pool.get("dx_a", (M, D))
            dqk = pool.get("d_qk", (M, 2 * D))
            # MLP
            wg(dx, h, w["gw3"], w["gb3"])
            for hh in range(S):
                with on(hh):
                    ops.linear_dgrad_swiglu(rs(dx, hh), w["pw3"], rs(x12, hh), rs(d_x12, hh), workspace=rs(d_h, hh))
            wg(d_x12, xn2, w["gw12"], w["gb12"])
            for hh in range(S):
                with on(hh):
                    ops.linear_dgrad(rs(d_x12, hh), w["pw12"], out=rs(d_b, hh))
                    ops.rmsnorm_bwd(rs(d_b, hh), rs(xm, hh), rs(rstd2, hh), w["pn2"], dres=rs(dx, hh),
                                    dx=rs(dx_b, hh), dw_part=part2[hh * nb_h:(hh + 1) * nb_h])
            dxm = dx_b
            # attention (norm2's weight gradient: its partial rows summed by the o-projection wgrad's reduce launch)
            ev_o = wg(dxm, o, w["gwo"], w["gbo"], rows_sum=(part2[:S * nb_h], w["gn2"], acc))
            for hh in range(S):
                with on(hh):
                    ops.linear_dgrad(rs(dxm, hh), w["pwo"], out=rs(d_o, hh))
            settle_qkv()  # d_qkv and the QK-norm partial rows are rewritten below
            if FUSED_QKNORM_BWD and n_i < rows and not pre_zeroed:
                # the context rows take no gradient in the blocks before context_start_block (the fused backward
                # writes rows < n_i only; the standalone QK-norm backward below zeroes them itself)
                dqkv.view(B, rows, 3 * D)[:, n_i:].zero_()
                pre_zeroed = True
            if FUSED_QKNORM_BWD:  # (S == 1)
                # attention backward with the QK-RMSNorm + RoPE backward fused into its dQ / dK stores: dqkv receives
                # the gradients of the raw q | k | v projections directly
                a5 = (ops._t4(qk, B, rows, Hh, 0), ops._t4(qk, B, rows, Hh, D), ops._t4(qkv, B, rows, Hh, 2 * D),
                      ops._t4(o, B, rows, Hh, 0), ops._t4(d_o, B, rows, Hh, 0), lse, delta, kbias)
                ops.attn_bwd_qknorm(*a5, ops._t4(qkv, B, rows, Hh, 0), ops._t4(qkv, B, rows, Hh, D),
                                    w["pqk_norm"][:64], w["pqk_norm"][64:], cos_t, sin_t, ops._t4(dqkv, B, rows, Hh, 0),
                                    ops._t4(dqkv, B, rows, Hh, D), qk_dw, ops._t4(dqkv, B, rows, Hh, 2 * D),
                                    B, Hh, rows, n_i, n_pre, scale)
                qk_job = (qk_dw[:ops.attn_bwd_dw_rows(B, Hh, n_i)], w["gqk_norm"], acc)
            else:
                for hh in range(S):
                    with on(hh):
                        qkh, qkvh, dqkh, dqkvh = rs(qk, hh), rs(qkv, hh), rs(dqk, hh), rs(dqkv, hh)
                        ops.attn_bwd(ops._t4(qkh, Bh, rows, Hh, 0), ops._t4(qkh, Bh, rows, Hh, D),
                                     ops._t4(qkvh, Bh, rows, Hh, 2 * D), ops._t4(rs(o, hh), Bh, rows, Hh, 0),
                                     ops._t4(rs(d_o, hh), Bh, rows, Hh, 0), bs(lse, hh), bs(delta, hh), bs(kbias, hh),
                                     ops._t4(dqkh, Bh, rows, Hh, 0), ops._t4(dqkh, Bh, rows, Hh, D),
                                     ops._t4(dqkvh, Bh, rows, Hh, 2 * D), Bh, Hh, rows, n_i, n_pre, scale,
                                     queue=ATTN_BWD_QUEUE)
                        # rows >= n_i (a pre-context block's context rows): zero q | k | v gradients, dqk not read there
                        ops.qknorm_rope_bwd(dqkh, qkvh, w["pqk_norm"][:64], w["pqk_norm"][64:], cos_t, sin_t, rows,
                                            dqkvh, dw_part=qkp[hh * nq_h:(hh + 1) * nq_h], n_valid=n_i)
                qk_job = (qkp[:S * nq_h], w["gqk_norm"], acc)
            ev_qkv = wg(dqkv, xn1, w["gwqkv"], w["gbqkv"], rows_sum=qk_job)
            for hh in range(S):
                with on(hh):
                    ops.linear_dgrad(rs(dqkv, hh), w["pwqkv"], out=rs(d_b, hh))
            settle(ev_o)  # the MLP / o-projection wgrads read dx_a, dx_b and part2, rewritten from here on
            for hh in range(S):
                with on(hh):
                    ops.rmsnorm_bwd(rs(d_b, hh), rs(x_in, hh), rs(rstd1, hh), w["pn1"], dres=rs(dxm, hh),
                                    dx=rs(dx_a, hh), dw_part=part1[hh * nb_h:(hh + 1) * nb_h])
            if S == 1:
                ops.reduce_rows(part1[:nb_h], w["gn1"], acc)
            else:  # over every lane's partial rows: on the side stream, after all lanes
                side_wait()
                with torch.cuda.stream(side):
                    ops.reduce_rows(part1[:S * nb_h], w["gn1"], acc)
                ev_qkv = torch.cuda.Event()
                ev_qkv.record(side)
            if side is None:
                if on_ready is not None:
                    on_ready(f"block{i}")  # every blocks.{i}.* gradient is enqueued
            else:
                ready = f"block{i}"  # announced at the next settle_qkv(), after its last side-stream launch
            dx = dx_a
            if n_ctx and self._ctx_refresh(i):
                for hh in range(S):
                    with on(hh):
                        r0 = hh * Bh * n_ctx
                        ops.ctx_rows(rs(dx, hh), Bh, n_pre, rows, n_ctx, dctx=dctx[r0:r0 + Bh * n_ctx],
                                     backward=True, overwrite=not dctx_set)
                dctx_set = True
        settle_qkv()
        if S > 1:
            for ln in lanes:
                main.wait_stream(ln)
        self._wait_inputs = None
        if side is not None:
            # the embeddings' small GEMMs reuse their gradient buffers back to back (d_h1 / d_a1 per embedder): they
            # run on the main stream, after every block's weight gradient
            main.wait_stream(side)
            on_side = False
        # --- embeddings backward
        dpe2 = pool.get("d_pe2", (M2, D))
        dsize = pool.get("d_size", (6 * B, D))
        dtime = pool.get("d_time", (B, D))
        ops.disassemble_tokens(dx, B, np_, rows, dpe2, dsize, dtime, self._tpe_grad_target(acc))
        if acc:
            self.g["time_position_embeds"].add_(pool.get("dtpe_tmp", (self.T, D), F32))
        bd = cfg.bottleneck_dim
        pe1 = pool.get("pe1", (M2, bd))
        wgrad(dpe2, pe1, g["patch_embedder.proj_2.weight"], g["patch_embedder.proj_2.bias"])
        dpe1 = ops.linear_dgrad(dpe2, self.p["patch_embedder.proj_2.weight"].view(D, bd), out=pool.get("d_pe1", (M2, bd)))
        wgrad(dpe1, st["zp"], g["patch_embedder.proj_1.weight"])
        for pre, rowsn, dy in (("time_embedder", B, dtime), ("image_size_embedder", 6 * B, dsize)):
            k = "t" if pre == "time_embedder" else "s"
            a1, h1 = pool.get(k + "_a1", (rowsn, D)), pool.get(k + "_h1", (rowsn, D))
            emb_in = pool.get(("temb_in" if k == "t" else "semb_in"), (rowsn, 256))
            wgrad(dy, h1, g[pre + ".mlp.2.weight"], g[pre + ".mlp.2.bias"])
            dh1 = ops.linear_dgrad(dy, self.p[pre + ".mlp.2.weight"], out=pool.get("d_h1", (rowsn, D)))
            da1 = ops.silu_bwd(dh1, a1, pool.get("d_a1", (rowsn, D)))
            wgrad(da1, emb_in, g[pre + ".mlp.0.weight"], g[pre + ".mlp.0.bias"])
        dctx_raw = None
        if n_ctx and not dctx_set:
            dctx.zero_()  # no refresh block (not reached for a context that enters at a block)
        if n_ctx:
            dctx_b = ops.cast_f32_bf16(dctx, pool.get("dctx_bf16", (B * n_ctx, D)))
            wgrad(dctx_b, st["ctx_raw"], g["context_embedder.weight"], g["context_embedder.bias"])
            dctx_raw = ops.linear_dgrad(dctx_b, self.p["context_embedder.weight"],
                                        out=pool.get("d_ctx_raw", (B * n_ctx, cfg.context_dim)))
        return dctx_raw

    def _zero_unwritten_grads(self, n_ctx: int, overwritten: tuple = ()):
        names = ["class_encoder.embedding.weight"]
        if not n_ctx:
            names += ["context_embedder.weight", "context_embedder.bias"]
        for n in names:
            if n in self.g and n not in overwritten:
                self.g[n].zero_()

    def _tpe_grad_target(self, acc: bool):
        if acc:
            return self.pool.get("dtpe_tmp", (self.T, self.D), F32)
        return self.g["time_position_embeds"]

    def _ws_elems(self, M: int) -> int:
        """f32 elements of the wgrad workspace: the largest split-K slab set + per-split bias sums (or the
        colsum partials of the non-ring fallback) over the engine's weight-gradient shapes."""
        D, F = self.D, self.F
        best = 1
        for N, K in ((D, F), (2 * F, D), (3 * D, D), (D, D), (self.fin["pwl"].shape[0], D)):
            s = ops.wgrad_splits(N, K, M) * WGRAD_SPLIT_MUL
            best = max(best, ops.linear_wgrad_workspace_bytes(M, N, K, s) // 4 + 1)
        return best
