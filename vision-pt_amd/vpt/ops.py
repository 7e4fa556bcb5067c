"""Tensor-level wrappers over the C-ABI kernels (plumbing only: PyTorch provides device memory
and the current HIP stream; every FLOP runs in libvpt_hip.so).

Conventions: bf16 activations/weights, f32 statistics and gradients-of-weights. Matrices are
row-major with an explicit leading dimension (`t.stride(0)`); the last dim must be contiguous.
"""

from __future__ import annotations

import contextlib
import ctypes

import torch

from . import _lib
from ._lib import call  # the size helpers read _lib.lib per call: tools/ may switch builds (use_library)

BF16 = torch.bfloat16
F32 = torch.float32

OUT_BF16, OUT_F32, OUT_F32_ACC = 0, 1, 2
ACT_NONE, ACT_SILU = 0, 1


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class KernelProbe:
    """Brackets every launch of one op with HIP events on the launching stream (used by bench.py
    to time the dominant kernel inside the timed region). `flops_fn(**shape)` gives the
    algorithmic FLOPs of one launch."""

    def __init__(self, op: str):
        self.op = op
        self.records: list[tuple] = []
        self.nbytes: list[float] = []
        self.active = False

    def record(self, flops: float, fn, key=None, nbytes: float = 0.0):
        """nbytes: compulsory HBM bytes of the launch (operands read once, results written once)."""
        if not self.active:
            return fn()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.records.append((s, e, flops, key))
        self.nbytes.append(nbytes)
        return r

    def mean_bytes(self) -> float:
        return sum(self.nbytes) / len(self.nbytes) if self.nbytes else 0.0

    def summary(self):
        """(launches, mean ms per launch, mean algorithmic FLOPs per launch)."""
        if not self.records:
            return 0, 0.0, 0.0
        ms = [r[0].elapsed_time(r[1]) for r in self.records]
        fl = [r[2] for r in self.records]
        return len(ms), sum(ms) / len(ms), sum(fl) / len(fl)

    def by_key(self):
        """{key: (launches, total ms, total algorithmic work)} over the keyed launches."""
        out: dict = {}
        for s, e, f, k in self.records:
            n, t, w = out.get(k, (0, 0.0, 0.0))
            out[k] = (n + 1, t + s.elapsed_time(e), w + f)
        return out


PROBES: dict[str, KernelProbe] = {}


def _launch(op: str, work: float, run):
    """Runs `run`; when a probe for `op` is active, brackets it with HIP events and records `work`
    (algorithmic FLOPs for MFMA ops, algorithmic HBM bytes for the memory-bound ones)."""
    pr = PROBES.get(op)
    if pr is None:
        return run()
    return pr.record(work, run)


def _p(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def _chk(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dim")


# ----------------------------------------------------------------------------- GEMM
def gemm(a, a_kmajor: bool, b, b_kmajor: bool, M: int, N: int, K: int, out, *, bias=None, resid=None,
         out_mode=OUT_BF16, act=ACT_NONE, splits=1, workspace=None, alpha=1.0, geometry=0, ring_grid=0):
    """out[M,N] (=|+=) alpha * sum_k A(m,k) B(n,k) (+bias[n]) (+resid[m,n]); see csrc/gemm.hip.
    geometry / ring_grid (0 = automatic) force a tile geometry per call (vpt_gemm_bf16_tiled)."""
    _chk(a, BF16, "a")
    _chk(b, BF16, "b")
    _chk(out, BF16 if out_mode == OUT_BF16 else F32, "out")
    if bias is not None:
        _chk(bias, BF16, "bias")
    if resid is not None:
        _chk(resid, BF16, "resid")
    if splits > 1 and workspace is None:
        workspace = torch.empty(splits * M * N, dtype=F32, device=out.device)

    args = (a.data_ptr(), a.stride(0), int(a_kmajor), b.data_ptr(), b.stride(0), int(b_kmajor), out.data_ptr(),
            out.stride(0), M, N, K, _p(bias), _p(resid), 0 if resid is None else resid.stride(0), out_mode, act, splits,
            _p(workspace), float(alpha))

    def run():
        if geometry or ring_grid:
            call("vpt_gemm_bf16_tiled", *args, int(geometry), int(ring_grid), stream())
        else:
            call("vpt_gemm_bf16", *args, stream())
    pr = PROBES.get("gemm")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * N * K, run, key=f"{'fwd' if a_kmajor and b_kmajor else 'dgrad' if a_kmajor else 'wgrad'}"
                  f" M{M} N{N} K{K} s{splits}",
                  nbytes=2.0 * (M + N) * K + M * N * (2 if out_mode == OUT_BF16 else 4 if out_mode == OUT_F32 else 8)
                  + (2.0 * M * N if resid is not None else 0.0))
    return out


_WS: dict = {}  # (device, tag) -> f32 workspace grown on demand (stream-ordered reuse on one stream)


def workspace(dev, tag: str, n: int, dtype=F32) -> torch.Tensor:
    """A per-(device, tag) buffer of at least n elements, grown on demand (stream-ordered reuse)."""
    buf = _WS.get((str(dev), tag))
    if buf is None or buf.numel() < n or buf.dtype != dtype:
        buf = _WS[(str(dev), tag)] = torch.empty(n, dtype=dtype, device=dev)
    return buf[:n]


_TICKETS: dict = {}  # (device, stream) -> zero-filled u32 tickets of the in-launch row-block reductions


def tickets(dev, n: int) -> torch.Tensor:
    """Row-block tickets for a kernel whose in-launch reduction counts blocks on them (vpt_geglu_bwd_lora /
    vpt_geglu_fwd_lora): zero when allocated, left zero by every launch, so one buffer serves every shape; one per
    (device, current stream), so launches on one stream reuse it in order and two streams never share tickets."""
    key = (str(dev), stream())
    buf = _TICKETS.get(key)
    if buf is None or buf.numel() < n:
        buf = _TICKETS[key] = torch.zeros(max(n, 1024), dtype=torch.int32, device=dev)
    return buf


GEO_R2_128 = 1281  # 128 x 128 tiles on the R2 ring's pipeline (include/vpt_hip.h vpt_gemm_bf16_tiled)
LORA_R2_128 = True  # lora_gemm_plan: GEO_R2_128 instead of the two-stage 128 x 128 kernel (A/B knob)


def lora_gemm_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(geometry, splits) for a base+LoRA GEMM: the 256 x 256 ring when its tiles fill the chip (>= 160), a
    K-split ring for small grids over a long reduction (K >= 4096: ~240 work items), otherwise 128 x 128 tiles
    (2 blocks per CU; on the R2 pipeline with LORA_R2_128). Measured at the config-5 shapes (tools/c5_gemm_shapes.py,
    profiles/r03/; tools/c5_geometry_probe.py, profiles/r06/)."""
    t256 = ((M + 255) // 256) * ((N + 255) // 256)
    if t256 >= 160:
        return 256, 1
    if K >= 4096:
        sp = max(2, min(4, round(240 / t256), K // 1024))
        return 256, sp
    return (GEO_R2_128 if LORA_R2_128 else 128), 1


def gemm_lora(a, b, b_kmajor: bool, a2, b2, M: int, N: int, K: int, out, *, bias=None, resid=None, geometry=None,
              splits=None, alpha: float = 1.0, alpha_cols: int = 0):
    """out[M,N] = A . B (+bias) (+resid) + a2 . B2 with one rounding (vpt_gemm_bf16_lora): the base GEMM of a
    LoRALinear with its adapter term as a K-extension. Forward: a = x [M,K], b = W [N,K] (b_kmajor), a2 = ds [M,r],
    b2 = up [N,r]; input gradient: a = dy [M,N_out] (K = N_out), b = W [N_out, K_in] (not b_kmajor, N = K_in),
    a2 = vs [M,r], b2 = down [r, K_in]. alpha != 1: the f32 result of columns [0, alpha_cols) (all when 0) times alpha
    before the rounding (vpt_gemm_bf16_lora_scaled; no K split)."""
    for t, n in ((a, "a"), (b, "b"), (a2, "a2"), (b2, "b2")):
        _chk(t, BF16, n)
    _chk(out, BF16, "out")
    if bias is not None:
        _chk(bias, BF16, "bias")
    if resid is not None:
        _chk(resid, BF16, "resid")
    K2 = a2.shape[1]
    geo, sp = lora_gemm_plan(M, N, K)
    geometry = geo if geometry is None else geometry
    splits = sp if splits is None else splits
    scaled = alpha != 1.0
    if scaled:
        splits = 1
    ws = workspace(out.device, "gemm_lora", splits * M * N) if splits > 1 else None

    def run():
        if scaled:
            call("vpt_gemm_bf16_lora_scaled", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), int(b_kmajor),
                 a2.data_ptr(), a2.stride(0), b2.data_ptr(), b2.stride(0), K2, out.data_ptr(), out.stride(0), M, N, K,
                 _p(bias), _p(resid), 0 if resid is None else resid.stride(0), int(geometry), float(alpha),
                 int(alpha_cols), stream())
            return
        call("vpt_gemm_bf16_lora", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), int(b_kmajor), a2.data_ptr(),
             a2.stride(0), b2.data_ptr(), b2.stride(0), K2, out.data_ptr(), out.stride(0), M, N, K, _p(bias), _p(resid),
             0 if resid is None else resid.stride(0), OUT_BF16, int(splits), _p(ws), int(geometry), stream())
    pr = PROBES.get("gemm_lora")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * N * (K + K2), run, key=f"{'fwd' if b_kmajor else 'dgrad'} M{M} N{N} K{K}")
    return out


def gemm_lora_grouped(x, w_stacked, a2, ups, out, *, bias=None, resid=None, geometry=None, splits=None,
                      alpha: float = 1.0, alpha_cols: int = 0):
    """G LoRA targets reading x as one GEMM (vpt_gemm_bf16_lora_grouped): out[:, g*n:(g+1)*n] = x . W_g^T +
    a2[:, g*r:(g+1)*r] . ups[g]^T, W_g = w_stacked[g*n:(g+1)*n] (the dequantised bases side by side). alpha != 1:
    columns [0, alpha_cols) (all when 0) times alpha before the rounding (vpt_gemm_bf16_lora_grouped_scaled)."""
    for t, n in ((x, "x"), (w_stacked, "w_stacked"), (a2, "a2"), (out, "out")):
        _chk(t, BF16, n)
    G = len(ups)
    for u in ups:
        _chk(u, BF16, "up")
        if not u.is_contiguous():
            raise ValueError("ups must be contiguous [n, r]")
    M, K = x.shape
    gn, r = ups[0].shape
    geo, sp = lora_gemm_plan(M, G * gn, K)
    geometry = geo if geometry is None else geometry
    splits = sp if splits is None else splits
    scaled = alpha != 1.0
    if scaled:
        splits = 1
    ws = workspace(out.device, "gemm_lora", splits * M * G * gn) if splits > 1 else None
    ptrs = (ctypes.c_void_p * G)(*[u.data_ptr() for u in ups])

    def run():
        if scaled:
            call("vpt_gemm_bf16_lora_grouped_scaled", x.data_ptr(), x.stride(0), w_stacked.data_ptr(),
                 w_stacked.stride(0), a2.data_ptr(), a2.stride(0), ctypes.cast(ptrs, ctypes.c_void_p), G, r,
                 out.data_ptr(), out.stride(0), M, gn, K, _p(bias), _p(resid), 0 if resid is None else resid.stride(0),
                 int(geometry), float(alpha), int(alpha_cols), stream())
            return
        call("vpt_gemm_bf16_lora_grouped", x.data_ptr(), x.stride(0), w_stacked.data_ptr(), w_stacked.stride(0),
             a2.data_ptr(), a2.stride(0), ctypes.cast(ptrs, ctypes.c_void_p), G, r, out.data_ptr(), out.stride(0), M, gn,
             K, _p(bias), _p(resid), 0 if resid is None else resid.stride(0), int(splits), _p(ws), int(geometry),
             stream())
    pr = PROBES.get("gemm_lora")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * G * gn * (K + r), run, key=f"fwd{G} M{M} N{G * gn} K{K}")
    return out


def gemm_lora_stacked(x, w_stacked, a2, ups_stacked, g_n: int, out, *, geometry=None, splits=None):
    """G = ups_stacked.shape[0] / g_n LoRA targets over one input as one GEMM (vpt_gemm_bf16_lora_stacked):
    out[:, g*g_n:(g+1)*g_n] = x . W_g^T + a2[:, g*r:(g+1)*r] . up_g^T with W, up stacked by rows."""
    for t, n in ((x, "x"), (w_stacked, "w_stacked"), (a2, "a2"), (ups_stacked, "ups_stacked"), (out, "out")):
        _chk(t, BF16, n)
    M, K = x.shape
    NG, r = ups_stacked.shape
    G = NG // g_n
    if G * g_n != NG or w_stacked.shape[0] != NG or ups_stacked.stride(0) != r:
        raise ValueError("gemm_lora_stacked: stacked shapes")
    geo, sp = lora_gemm_plan(M, NG, K)
    geometry = geo if geometry is None else geometry
    splits = sp if splits is None else splits
    ws = workspace(out.device, "gemm_lora", splits * M * NG) if splits > 1 else None

    def run():
        call("vpt_gemm_bf16_lora_stacked", x.data_ptr(), x.stride(0), w_stacked.data_ptr(), w_stacked.stride(0),
             a2.data_ptr(), a2.stride(0), ups_stacked.data_ptr(), G, r, out.data_ptr(), out.stride(0), M, g_n, K,
             int(splits), _p(ws), int(geometry), stream())
    pr = PROBES.get("gemm_lora")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * NG * (K + r), run, key=f"stacked{G} M{M} N{NG} K{K}")
    return out


def linear(x, w, bias=None, resid=None, out=None, act=ACT_NONE, **tile):
    """y = x @ w.T (+bias) (+resid) in bf16 — nn.Linear forward."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=BF16, device=x.device)
    return gemm(x, True, w, True, M, N, K, out, bias=bias, resid=resid, act=act, **tile)


def linear_qknorm_rope(x, w, bias, qkv, qk, wq, wk, cos_t, sin_t, rows_per_seq, q_scale=1.0, eps=1e-6):
    """qkv = x @ w.T + bias (bf16, [M, 3D]) and qk = (rope(rms(q)) * q_scale | rope(rms(k))) [M, 2D] in ONE ring GEMM
    (vpt_linear_qknorm_rope: the norm + RoPE in the epilogue) -- what linear + qknorm_rope_fwd compute, bitwise."""
    M, K = x.shape
    N = w.shape[0]
    D = N // 3
    for t, n in ((x, "x"), (w, "w"), (qkv, "qkv"), (qk, "qk"), (wq, "wq"), (wk, "wk")):
        _chk(t, BF16, n)
    if bias is not None:
        _chk(bias, BF16, "bias")

    def run():
        call("vpt_linear_qknorm_rope", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), _p(bias), qkv.data_ptr(),
             qkv.stride(0), qk.data_ptr(), qk.stride(0), M, D, K, wq.data_ptr(), wk.data_ptr(), cos_t.data_ptr(),
             sin_t.data_ptr(), rows_per_seq, float(eps), float(q_scale), stream())
    pr = PROBES.get("gemm")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * N * K, run, key=f"fwd+qkn M{M} N{N} K{K} s1",
                  nbytes=2.0 * (M + N) * K + M * N * 2 + M * 2 * D * 2)
    return qkv, qk


def linear_dgrad(dy, w, out=None, resid=None, **tile):
    """dx = dy @ w (+resid) (dy [M,N], w [N,K]) — nn.Linear input gradient (resid: a second bf16 gradient
    of the same input, summed with the reference's bf16 rounding)."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=BF16, device=dy.device)
    return gemm(dy, True, w, False, M, K, N, out, resid=resid, **tile)


def linear_wgrad_workspace_bytes(M: int, N: int, K: int, splits: int) -> int:
    return int(call("vpt_linear_wgrad_workspace_bytes", M, N, K, splits))


def linear_wgrad(dy, x, out, accumulate=False, splits=1, workspace=None, bias_out=None, geometry=0, ring_grid=0,
                 rows_sum=None):
    """dW (=|+=) dy.T @ x in f32 (dy [M,N], x [M,K], out [N,K]) — nn.Linear weight gradient — and, with
    bias_out [N] f32, the bias gradient (=|+=) column sums of dy in the same ring GEMM (vpt_linear_wgrad).
    rows_sum = (part [R, C] f32, out [C] f32, accumulate): an unrelated reduce_rows job done by extra blocks of the
    weight gradient's reduce launch (vpt_linear_wgrad_rr) instead of a launch of its own."""
    M, N = dy.shape
    K = x.shape[1]
    _chk(dy, BF16, "dy")
    _chk(x, BF16, "x")
    _chk(out, F32, "out")
    if bias_out is not None:
        _chk(bias_out, F32, "bias_out")
        if not bias_out.is_contiguous() or bias_out.numel() != N:
            raise ValueError("bias_out must be a contiguous [N] f32 tensor")
    need = linear_wgrad_workspace_bytes(M, N, K, splits)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty((need + 3) // 4, dtype=F32, device=dy.device)

    if rows_sum is not None:
        rp, ro, racc = rows_sum
        _chk(rp, F32, "rows_sum part")
        _chk(ro, F32, "rows_sum out")
        if not rp.is_contiguous() or rp.dim() != 2 or ro.numel() != rp.shape[1] or not ro.is_contiguous():
            raise ValueError("rows_sum: part [R, C] and out [C], contiguous f32")

    def run():
        if rows_sum is None:
            call("vpt_linear_wgrad", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(),
                 out.stride(0), _p(bias_out), M, N, K, int(accumulate), splits, workspace.data_ptr(), int(geometry),
                 int(ring_grid), stream())
        else:
            call("vpt_linear_wgrad_rr", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(),
                 out.stride(0), _p(bias_out), M, N, K, int(accumulate), splits, workspace.data_ptr(), int(geometry),
                 int(ring_grid), rp.data_ptr(), rp.shape[0], rp.shape[1], ro.data_ptr(), int(racc), stream())
    pr = PROBES.get("gemm")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * N * K, run, key=f"wgrad M{N} N{K} K{M} s{splits}{' +b' if bias_out is not None else ''}",
                  nbytes=2.0 * M * (N + K) + N * K * (8 if accumulate else 4))
    return out


def linear_swiglu(x, w12, b12, x12, h):
    """x12 = x @ w12.T + b12 and h = bf16(silu(x1)) * x2 (SwiGLU, denoiser.py:480-506) in one GEMM."""
    M, K = x.shape
    F = w12.shape[0] // 2
    for t, n in ((x, "x"), (w12, "w12"), (x12, "x12"), (h, "h")):
        _chk(t, BF16, n)

    def run():
        call("vpt_gemm_swiglu_fwd", x.data_ptr(), x.stride(0), w12.data_ptr(), w12.stride(0), _p(b12), x12.data_ptr(),
             x12.stride(0), h.data_ptr(), h.stride(0), M, F, K, stream())
    pr = PROBES.get("gemm")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * 2 * F * K, run, key=f"swiglu_fwd M{M} N{2 * F} K{K}",
                  nbytes=2.0 * (M + 2 * F) * K + 2.0 * M * 3 * F)  # x12 and h out
    return x12, h


def linear_dgrad_swiglu(dy, w3, x12, dx12, workspace=None):
    """dx12 = SwiGLU backward of (dy @ w3) against x12 (dh stays in registers on the fused path)."""
    M, D = dy.shape
    F = w3.shape[1]
    for t, n in ((dy, "dy"), (w3, "w3"), (x12, "x12"), (dx12, "dx12")):
        _chk(t, BF16, n)
    need = int(call("vpt_gemm_swiglu_bwd_workspace", M, F, D))
    if need and (workspace is None or workspace.numel() * workspace.element_size() < need):
        workspace = torch.empty(M * F, dtype=BF16, device=dy.device)

    def run():
        call("vpt_gemm_swiglu_bwd", dy.data_ptr(), dy.stride(0), w3.data_ptr(), w3.stride(0), x12.data_ptr(),
             x12.stride(0), dx12.data_ptr(), dx12.stride(0), M, F, D, _p(workspace) if need else None, stream())
    pr = PROBES.get("gemm")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * F * D, run, key=f"swiglu_dgrad M{M} N{F} K{D}",
                  nbytes=2.0 * (M + F) * D + 2.0 * M * 2 * F * 2)  # x12 in, dx12 out
    return dx12


def wgrad_splits(N: int, K: int, M: int) -> int:
    """Split-K factor for a weight gradient dW[N,K] = dy[M,N]^T x[M,K] (reduction over M tokens).

    Cost model for the 256x256 ring kernel (one block per CU, 256 CUs): the tile grid runs in
    ceil(tiles*s/256) rounds of M/s tokens each (~33 ns per token per tile at ~1 PF/s chip-wide, plus
    ~3 us prologue/epilogue), and the split-K reduction streams s*N*K*4 bytes (~4 TB/s, ~5 us launch).
    """
    tiles = ((N + 255) // 256) * ((K + 255) // 256)
    best_s, best_t = 1, None
    for s in range(1, 65):
        if s > 1 and M // s < 256:
            break
        rounds = -(-tiles * s // 256)
        t = rounds * ((M / s) * 0.0336 + 3.0)
        if s > 1:
            t += (s + 1) * N * K * 4 / 4.0e6 + 5.0
        if best_t is None or t < best_t:
            best_s, best_t = s, t
    return best_s


# ----------------------------------------------------------------------------- norms
def rmsnorm_fwd(x, w, out=None, rstd=None, eps=1e-6):
    M, D = x.shape
    if out is None:
        out = torch.empty(M, D, dtype=BF16, device=x.device)
    if rstd is None:
        rstd = torch.empty(M, dtype=F32, device=x.device)
    _launch("rmsnorm_fwd", M * D * 4 + M * 4,  # bf16 x in, bf16 y out, f32 rstd
            lambda: call("vpt_rmsnorm_fwd", x.data_ptr(), x.stride(0), w.data_ptr(), out.data_ptr(), out.stride(0),
                         rstd.data_ptr(), M, D, eps, stream()))
    return out, rstd


def rmsnorm_bwd_blocks(M: int) -> int:
    return _lib.lib.vpt_rmsnorm_bwd_blocks(M)


def rmsnorm_bwd(dy, x, rstd, w, dres=None, dx=None, dw_part=None):
    """dx = dres + RMSNorm'(dy); dw_part [blocks, D] f32 partial sums (reduce with reduce_rows)."""
    M, D = x.shape
    if dx is None:
        dx = torch.empty(M, D, dtype=BF16, device=x.device)
    if dw_part is None:
        dw_part = torch.empty(rmsnorm_bwd_blocks(M), D, dtype=F32, device=x.device)
    nbytes = M * D * (6 + (2 if dres is not None else 0)) + M * 4 + dw_part.numel() * 4  # dy, x, (dres) in; dx out
    _launch("rmsnorm_bwd", nbytes,
            lambda: call("vpt_rmsnorm_bwd", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), rstd.data_ptr(),
                         w.data_ptr(), _p(dres), 0 if dres is None else dres.stride(0), dx.data_ptr(), dx.stride(0),
                         dw_part.data_ptr(), M, D, stream()))
    return dx, dw_part


def reduce_rows(part, out, accumulate=False):
    R, Cc = part.shape
    call("vpt_reduce_rows", part.data_ptr(), R, Cc, out.data_ptr(), int(accumulate), stream())
    return out


def qknorm_rope_fwd(qkv, wq, wk, cos_t, sin_t, rows_per_seq, out=None, eps=1e-6, q_scale=1.0):
    """qkv [M, 3D] -> out [M, 2D] = (rope(rms(q)) * q_scale, rope(rms(k))); q_scale = attn_q_scale() makes
    the q half the pre-scaled query the attention kernels take."""
    M = qkv.shape[0]
    D = qkv.shape[1] // 3
    if out is None:
        out = torch.empty(M, 2 * D, dtype=BF16, device=qkv.device)
    _launch("qknorm_rope_fwd", M * 2 * D * 4,  # q, k bf16 in and out (the RoPE table is L2-resident)
            lambda: call("vpt_qknorm_rope_fwd", qkv.data_ptr(), qkv.stride(0), wq.data_ptr(), wk.data_ptr(),
                         cos_t.data_ptr(), sin_t.data_ptr(), out.data_ptr(), out.stride(0), M, rows_per_seq, D, eps,
                         float(q_scale), stream()))
    return out


def qknorm_rope_blocks(M: int) -> int:
    return _lib.lib.vpt_qknorm_rope_blocks(M)


def qknorm_rope_bwd(dqk, qkv, wq, wk, cos_t, sin_t, rows_per_seq, dqkv, dw_part=None, eps=1e-6, n_valid=None):
    """Writes dqkv[:, :2D]; dw_part [blocks, 128] = (d q_norm.w | d k_norm.w) partials. n_valid < rows_per_seq: the
    rows past it get zero q | k | v gradients (dqk not read there)."""
    M = qkv.shape[0]
    D = qkv.shape[1] // 3
    nv = rows_per_seq if n_valid is None else n_valid
    if dw_part is None:
        dw_part = torch.empty(qknorm_rope_blocks(M), 128, dtype=F32, device=qkv.device)
    _launch("qknorm_rope_bwd", M * 2 * D * 6,  # dq, dk and q, k in; dq, dk out (bf16)
            lambda: call("vpt_qknorm_rope_bwd_rows", dqk.data_ptr(), dqk.stride(0), qkv.data_ptr(), qkv.stride(0),
                         wq.data_ptr(), wk.data_ptr(), cos_t.data_ptr(), sin_t.data_ptr(), dqkv.data_ptr(),
                         dqkv.stride(0), dw_part.data_ptr(), M, rows_per_seq, nv, D, eps, stream()))
    return dw_part


# ----------------------------------------------------------------------------- attention
def _t4(t, B: int, rows: int, H: int, col0: int = 0):
    """Token-major [B*rows, ld] matrix viewed per head: returns (ptr, sb, sh, sr) for head 0 at col0."""
    ld = t.stride(0)
    return t.data_ptr() + col0 * t.element_size(), rows * ld, 64, ld


def attn_q_scale(scale=0.125) -> float:
    """Factor the attention kernels expect pre-applied to q (scale * log2 e; see include/vpt_hip.h)."""
    return float(call("vpt_attn_q_scale", scale))


def attn_fwd(q, k, v, o, lse, kbias, B, H, rows, n, n_dense, scale=0.125, nk=None):
    """q/k/v/o as (ptr, sb, sh, sr) tuples (element strides); q PRE-SCALED by attn_q_scale(scale);
    lse [B,H,rows] f32 (receives -LSE in log2 units); kbias [B,keys] f32 or None; n query rows, nk key rows
    (default n; cross-attention otherwise)."""
    nk = n if nk is None else nk

    def run():
        call("vpt_attn_fwd", *q, *k, *v, *o, lse.data_ptr(), lse.stride(0), lse.stride(1),
             _p(kbias), 0 if kbias is None else kbias.stride(0), B, H, n, nk, n_dense, scale, stream())
    pr = PROBES.get("attn_fwd")
    if pr is None:
        return run()
    # compulsory: q, o (n rows), k, v (nk rows) bf16 of 64 dims, -LSE f32
    return pr.record(4.0 * B * H * n * nk * 64, run, nbytes=B * H * (2.0 * 64 * 2 * (n + nk) + 4.0 * n))


def attn_fwd_qknorm(q, k, v, o, lse, kbias, wq, wk, B, H, rows, n, n_dense, scale=0.125):
    """attn_fwd for QK-RMSNormed self-attention inputs (include/vpt_hip.h vpt_attn_fwd_qknorm): a fixed softmax
    reference point from the norm weights wq / wk [64] instead of the running row maximum."""
    def run():
        call("vpt_attn_fwd_qknorm", *q, *k, *v, *o, lse.data_ptr(), lse.stride(0), lse.stride(1),
             _p(kbias), 0 if kbias is None else kbias.stride(0), wq.data_ptr(), wk.data_ptr(), B, H, n, n, n_dense,
             scale, stream())
    pr = PROBES.get("attn_fwd")
    if pr is None:
        return run()
    return pr.record(4.0 * B * H * n * n * 64, run, nbytes=B * H * (2.0 * 64 * 2 * (2 * n) + 4.0 * n))


_ATTN_QUEUES: dict = {}


def attn_queue(device=None) -> torch.Tensor:
    """The persistent backward's 64-byte work-queue words for the current stream (zeroed once; every launch leaves
    them zero): one set per stream, since launches on different streams may overlap."""
    st = torch.cuda.current_stream(device)
    key = (st.device.index, st.cuda_stream)
    ws = _ATTN_QUEUES.get(key)
    if ws is None:
        ws = torch.zeros(int(_lib.lib.vpt_attn_bwd_queue_bytes()) // 4, dtype=torch.int32, device=st.device)
        _ATTN_QUEUES[key] = ws
    return ws


def attn_bwd(q, k, v, o, do, lse, delta, kbias, dq, dk, dv, B, H, rows, n, n_dense, scale=0.125, nk=None,
             queue=False):
    """queue: the persistent work-queue kernel (vpt_attn_bwd_q, bitwise the same results) instead of one block per
    item (vpt_attn_bwd)."""
    nk = n if nk is None else nk
    ws = attn_queue() if queue else None

    def run():
        if ws is not None:
            call("vpt_attn_bwd_q", *q, *k, *v, *o, *do, lse.data_ptr(), delta.data_ptr(), lse.stride(0),
                 lse.stride(1), _p(kbias), 0 if kbias is None else kbias.stride(0), *dq, *dk, *dv, B, H, n, nk,
                 n_dense, scale, ws.data_ptr(), stream())
            return
        call("vpt_attn_bwd", *q, *k, *v, *o, *do, lse.data_ptr(), delta.data_ptr(), lse.stride(0), lse.stride(1),
             _p(kbias), 0 if kbias is None else kbias.stride(0), *dq, *dk, *dv, B, H, n, nk, n_dense, scale,
             stream())
    pr = PROBES.get("attn_bwd")
    if pr is None:
        return run()
    # compulsory: q, o, do read + dq written (n rows), k, v read + dk, dv written (nk rows), -LSE / -delta
    return pr.record(8.0 * B * H * n * nk * 64, run, nbytes=B * H * (2.0 * 64 * 4 * (n + nk) + 12.0 * n))


def attn_bwd_dw_rows(B: int, H: int, n: int) -> int:
    return int(_lib.lib.vpt_attn_bwd_dw_rows(B, H, n))


def attn_bwd_qknorm(q, k, v, o, do, lse, delta, kbias, xq, xk, wq, wk, cos_t, sin_t, dq, dk, dw_part, dv,
                    B, H, rows, n, n_dense, scale=0.125, eps=1e-6):
    """attn_bwd with the QK-RMSNorm + RoPE backward fused into the dQ / dK stores (include/vpt_hip.h
    vpt_attn_bwd_qknorm): xq / xk (raw projections) and dq / dk share their (sb, sh, sr) strides; dq / dk receive the
    raw-projection gradients; dw_part [>= attn_bwd_dw_rows(B, H, n), 128] f32 the q_norm | k_norm weight partials
    (one reduce_rows into the 128 weight gradients)."""
    if xq[1:] != xk[1:] or dq[1:] != dk[1:]:
        raise ValueError("attn_bwd_qknorm: q / k operands must share strides")
    rows_needed = attn_bwd_dw_rows(B, H, n)
    if dw_part.dtype != F32 or dw_part.dim() != 2 or dw_part.shape[0] < rows_needed or dw_part.shape[1] != 128 \
            or not dw_part.is_contiguous():
        raise ValueError(f"attn_bwd_qknorm: dw_part must be contiguous f32 [>= {rows_needed}, 128]")

    def run():
        call("vpt_attn_bwd_qknorm", *q, *k, *v, *o, *do, lse.data_ptr(), delta.data_ptr(), lse.stride(0), lse.stride(1),
             _p(kbias), 0 if kbias is None else kbias.stride(0), xq[0], xk[0], *xq[1:], wq.data_ptr(), wk.data_ptr(),
             cos_t.data_ptr(), sin_t.data_ptr(), float(eps), dq[0], dk[0], *dq[1:], dw_part.data_ptr(),
             dw_part.data_ptr() + 64 * 4, 128, *dv, B, H, n, n, n_dense, scale, stream())
    pr = PROBES.get("attn_bwd")
    if pr is None:
        return run()
    return pr.record(8.0 * B * H * n * n * 64, run, nbytes=B * H * (2.0 * 64 * 4 * (2 * n) + 12.0 * n))


# ----------------------------------------------------------------------------- misc
def patchify(img, B, H, W, out, t=None, noise=None, noise_scale=1.0, seed=0, noising=True):
    _launch("patchify", B * 3 * H * W * (4 + (2 if noise is not None else 0)),  # fp16 pixel in, bf16 out
            lambda: call("vpt_patchify", img.data_ptr(), 0 if noising else 1, _p(noise), _p(t), noise_scale, seed, B,
                         H, W, out.data_ptr(), stream()))
    return out


def gauss_noise(out, seed, noise_scale=1.0):
    """out (fp16, any shape, even numel) <- the in-kernel noise draw of `seed` at each flat element index."""
    call("vpt_gauss_noise", out.numel(), seed, noise_scale, out.data_ptr(), stream())
    return out


def area_lowres(img, B, H, W, k, t, img_lr, noise_lr, z_lr, noise=None, noise_scale=1.0, seed=0):
    """F.interpolate(mode="area", scale_factor=1/k) of the fp16 image, the fp16 noise (explicit or regenerated from
    `seed`) and the noisy image (arb_class_to_image.py:233-245) -> img_lr / noise_lr fp16, z_lr bf16 [B,3,H/k,W/k]."""
    _launch("area_lowres", B * 3 * H * W * (2 + (2 if noise is not None else 0)) + B * 3 * (H // k) * (W // k) * 6,
            lambda: call("vpt_area_lowres", img.data_ptr(), _p(noise), t.data_ptr(), noise_scale, seed, B, H, W, k,
                         img_lr.data_ptr(), noise_lr.data_ptr(), z_lr.data_ptr(), stream()))
    return img_lr, noise_lr, z_lr


def unpatchify(patches, B, H, W, img, reverse=False):
    call("vpt_unpatchify", patches.data_ptr(), B, H, W, img.data_ptr(), int(reverse), stream())
    return img


def euler_cfg_step(z, pred, B, H, W, cfg, cfg_scale, mode, t, dt):
    """z [B,3,H,W] bf16 (in place) <- Euler step from the patch-layout prediction (see vpt_euler_cfg_step)."""
    call("vpt_euler_cfg_step", z.data_ptr(), pred.data_ptr(), B, H, W, int(cfg), float(cfg_scale), int(mode),
         float(t), float(dt), stream())
    return z


def loss_blocks() -> int:
    return _lib.lib.vpt_loss_blocks()


def flow_loss(pred, img, t, B, H, W, dpred, part, loss, target=0, t_eps=0.05, noise=None, noise_scale=1.0,
              seed=0):
    _launch("flow_loss", B * 3 * H * W * (6 + (2 if noise is not None else 0)),  # pred, image in; dpred out
            lambda: call("vpt_flow_loss", pred.data_ptr(), img.data_ptr(), _p(noise), t.data_ptr(), noise_scale, seed,
                         target, t_eps, B, H, W, dpred.data_ptr(), part.data_ptr(), loss.data_ptr(), stream()))
    return loss


def timestep_embed(vals, out):
    call("vpt_timestep_embed", vals.data_ptr(), vals.numel(), out.data_ptr(), stream())
    return out


def assemble_tokens(patches, size_emb, time_emb, tpe, ctx, n_ctx, B, np_, rows, x):
    call("vpt_assemble_tokens", patches.data_ptr(), size_emb.data_ptr(), time_emb.data_ptr(), tpe.data_ptr(),
         _p(ctx), n_ctx, B, np_, rows, x.shape[1], x.data_ptr(), stream())
    return x


def disassemble_tokens(dx, B, np_, rows, dpatches, dsize, dtime, dtpe):
    call("vpt_disassemble_tokens", dx.data_ptr(), B, np_, rows, dx.shape[1], dpatches.data_ptr(), dsize.data_ptr(),
         dtime.data_ptr(), _p(dtpe), stream())


def ctx_rows(x, B, row0, rows, n_ctx, ctx=None, dctx=None, backward=False, overwrite=False):
    """Forward: ctx -> the context rows of x. Backward: those rows of x -> dctx (+=, or = with overwrite), then zeroed."""
    mode = (2 if overwrite else 1) if backward else 0
    call("vpt_ctx_rows", x.data_ptr(), B, row0, rows, x.shape[1], _p(ctx), _p(dctx), n_ctx, mode, stream())


def swiglu_fwd(x12, h):
    M, F2 = x12.shape
    call("vpt_swiglu_fwd", x12.data_ptr(), M, F2 // 2, h.data_ptr(), stream())
    return h


def swiglu_bwd(dh, x12, dx12):
    M, F2 = x12.shape
    call("vpt_swiglu_bwd", dh.data_ptr(), x12.data_ptr(), M, F2 // 2, dx12.data_ptr(), stream())
    return dx12


def colsum_blocks(M: int) -> int:
    return _lib.lib.vpt_colsum_blocks(M)


def bias_grad(dy, out, part=None, accumulate=False):
    """out[N] (=|+=) sum over rows of dy [M,N] (bf16) in f32 (slice partials + fixed-order row sum)."""
    M, N = dy.shape
    nb = colsum_blocks(M)
    if part is None:
        part = torch.empty(nb, N, dtype=F32, device=dy.device)
    part = part.view(-1)[: nb * N]
    _launch("bias_grad", M * N * 2 + nb * N * 8,  # dy read once; partials written and read back
            lambda: call("vpt_bias_grad", dy.data_ptr(), dy.stride(0), M, N, part.data_ptr(), out.data_ptr(),
                         int(accumulate), stream()))
    return out


def embed_gather(table, ids, out):
    R = ids.numel()
    if R == 0:  # a context-free batch (n_ctx = 0): nothing to gather
        return out
    call("vpt_embed_gather", table.data_ptr(), ids.data_ptr(), R, table.shape[1], out.data_ptr(), stream())
    return out


def embed_scatter_add(drows, ids, pad_id, dtable):
    R = ids.numel()
    if R == 0:
        return
    call("vpt_embed_scatter_add", drows.data_ptr(), ids.data_ptr(), R, dtable.shape[1], pad_id, dtable.data_ptr(),
         stream())


def embed_grad_set(drows, ids, pad_id, dtable, accumulate=False):
    """dtable[V, D] f32 = (or += with accumulate) the embedding gradient of drows [R, D] bf16 at ids [R]; overwrite:
    padding row and unnamed rows zero; each row summed in position order (deterministic on both paths)."""
    R = ids.numel()
    call("vpt_embed_grad_set", drows.data_ptr() if R else None, ids.data_ptr() if R else None, R, dtable.shape[1],
         pad_id, dtable.shape[0], int(bool(accumulate)), dtable.data_ptr(), stream())
    return dtable


EMBED_GRAD_SET_MAX_IDS = 16384


def step_inputs(t, tscale, orig, target, crop, t_vals, size_vals, mask, n_ctx, n_pre, rows, kbias):
    """vpt_step_inputs: t [B] f32, orig / target / crop int64 [B, 2] (device, contiguous), mask int64 [B, n_ctx] or
    None -> t_vals [B], size_vals [6B] f32 and kbias[:, :n_pre + n_ctx] (row stride rows)."""
    B = t.numel()
    call("vpt_step_inputs", t.data_ptr(), B, tscale, orig.data_ptr(), target.data_ptr(), crop.data_ptr(),
         t_vals.data_ptr(), size_vals.data_ptr(), None if mask is None else mask.data_ptr(), n_ctx, n_pre, rows,
         kbias.data_ptr(), stream())


def copy_rows(seq, rows, row0, cnt, dense, B, reverse=False, zero_rest=False):
    """dense[B*cnt, D] <-> seq[B*rows, D] rows [row0, row0+cnt) of every sequence; zero_rest (with reverse) also
    zeroes every other row of seq (one pass instead of a fill before the scatter)."""
    D = dense.shape[1]
    if zero_rest and not reverse:
        raise ValueError("copy_rows: zero_rest needs reverse=True")
    call("vpt_copy_rows", seq.data_ptr(), seq.stride(0), rows, row0, cnt, dense.data_ptr(), dense.stride(0), B, D,
         2 if zero_rest else int(reverse), stream())
    return dense


def silu(x, out):
    call("vpt_silu", x.data_ptr(), None, out.data_ptr(), x.numel(), 0, stream())
    return out


def silu_bwd(dy, x, dx):
    call("vpt_silu", x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), 1, stream())
    return dx


def cast_f32_bf16(x, out):
    call("vpt_cast_f32_bf16", x.data_ptr(), x.numel(), out.data_ptr(), stream())
    return out


def radam_sf_step(y, grad, z, v, *, beta2, bias_correction2, eps, ckp1, adaptive_y_lr, lr, decay, grad_scale,
                  adam, clip_coef=None, clip_value=0.0):
    """grad f32, or bf16 (the all-reduced bf16 wire buffer of vpt.ddp.GradSync); clip_coef = a device f32
    scalar multiplying the gradient (global-norm clipping), clip_value > 0 clamps it afterwards."""
    if grad.dtype not in (F32, BF16) or grad.numel() != y.numel():
        raise ValueError("grad must be f32 or bf16 with y's size")
    if clip_coef is not None:
        _chk(clip_coef, F32, "clip_coef")
    gb = grad.dtype == BF16
    _launch("radam_sf_step", y.numel() * (22 if gb else 24),  # y bf16, grad, z / v f32 in; y, z, v out
            lambda: call("vpt_radam_sf_step", y.data_ptr(), grad.data_ptr(), int(gb), z.data_ptr(), v.data_ptr(),
                         y.numel(),
                         beta2, bias_correction2, eps, ckp1, adaptive_y_lr, lr, decay, grad_scale, int(adam),
                         _p(clip_coef), float(clip_value or 0.0), stream()))


GRAD_NORM_BLOCKS = None


def grad_norm_blocks() -> int:
    global GRAD_NORM_BLOCKS
    if GRAD_NORM_BLOCKS is None:
        GRAD_NORM_BLOCKS = int(call("vpt_grad_norm_blocks"))
    return GRAD_NORM_BLOCKS


def grad_sumsq(g, scale, part):
    """part[grad_norm_blocks()] f32 <- partial sums of (scale * g)^2 (g f32 or bf16)."""
    if g.dtype not in (F32, BF16):
        raise ValueError("g must be f32 or bf16")
    _chk(part, F32, "part")
    if part.numel() < grad_norm_blocks():
        raise ValueError("part too small")
    call("vpt_grad_sumsq", g.data_ptr(), int(g.dtype == BF16), g.numel(), float(scale), part.data_ptr(), stream())


def clip_coef(part, max_norm, coef, norm_out=None):
    """coef (device f32 scalar) <- min(1, max_norm / (sqrt(sum(part)) + 1e-6)); norm_out <- the norm."""
    _chk(part, F32, "part")
    call("vpt_clip_coef", part.data_ptr(), part.numel(), float(max_norm), coef.data_ptr(), _p(norm_out), stream())


def sf_lerp(y, z, w):
    call("vpt_sf_lerp", y.data_ptr(), z.data_ptr(), y.numel(), w, stream())


def ema_update(ema, params, decay, first):
    # (1 - decay) is formed in Python double and only then rounded to f32, as torch rounds the Python scalar
    # of `(1 - decay) * p` (swa_utils.get_ema_avg_fn); 1 - float32(decay) differs by 1.7e-4 relative at 0.9999
    call("vpt_ema_update", ema.data_ptr(), params.data_ptr(), params.numel(), float(decay), float(1.0 - decay),
         int(first), stream())


def sf_init(y, z, v):
    call("vpt_sf_init", y.data_ptr(), z.data_ptr(), v.data_ptr(), y.numel(), stream())


# ----------------------------------------------------------------------------- SDXL block (a29, a30)
def layernorm_fwd(x, w, b, out=None, mean=None, rstd=None, eps=1e-5):
    M, D = x.shape
    out = torch.empty(M, D, dtype=BF16, device=x.device) if out is None else out
    mean = torch.empty(M, dtype=F32, device=x.device) if mean is None else mean
    rstd = torch.empty(M, dtype=F32, device=x.device) if rstd is None else rstd
    call("vpt_layernorm_fwd", x.data_ptr(), x.stride(0), w.data_ptr(), b.data_ptr(), out.data_ptr(), out.stride(0),
         mean.data_ptr(), rstd.data_ptr(), M, D, eps, stream())
    return out, mean, rstd


def layernorm_lora_fwd(x, w, b, down, G: int, alpha: float, ds, eps=1e-5):
    """layernorm_fwd and, in the same launch, ds[:, 16g:16g+16] = bf16(alpha * y . down_g^T) for g < G, down_g the
    g-th [16, D] block of `down` (the flat layout's adjacent downs; csrc/sdxl.hip layernorm_lora_fwd_kernel)."""
    M, D = x.shape
    _chk(down, BF16, "down")
    if down.stride(-1) != 1 or ds.stride(1) != 1 or ds.shape[1] < 16 * G:
        raise ValueError("layernorm_lora_fwd: row-major down / ds with 16 G columns")
    out = torch.empty(M, D, dtype=BF16, device=x.device)
    mean = torch.empty(M, dtype=F32, device=x.device)
    rstd = torch.empty(M, dtype=F32, device=x.device)
    call("vpt_layernorm_lora_fwd", x.data_ptr(), x.stride(0), w.data_ptr(), b.data_ptr(), out.data_ptr(), out.stride(0),
         mean.data_ptr(), rstd.data_ptr(), M, D, eps, down.data_ptr(), 16 * D, G, ds.data_ptr(), ds.stride(0),
         float(alpha), stream())
    return out, mean, rstd


def layernorm_bwd(dy, x, mean, rstd, w, dres=None, dx=None, dw_part=None, db_part=None):
    """dx = dres + LayerNorm'(dy); optional per-block dw/db partials [layernorm_bwd_blocks(M), D]."""
    M, D = x.shape
    dx = torch.empty(M, D, dtype=BF16, device=x.device) if dx is None else dx
    call("vpt_layernorm_bwd", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), mean.data_ptr(), rstd.data_ptr(),
         w.data_ptr(), _p(dres), 0 if dres is None else dres.stride(0), dx.data_ptr(), dx.stride(0), _p(dw_part),
         _p(db_part), M, D, stream())
    return dx


def layernorm_bwd_lora(dy, x, mean, rstd, w, up, alpha: float, vs, dres=None):
    """layernorm_bwd (no partials) and, in the same launch, vs = bf16(alpha * dx . up) (up [D, 16];
    csrc/sdxl.hip layernorm_bwd_lora_kernel). Returns dx."""
    M, D = x.shape
    _chk(up, BF16, "up")
    if not up.is_contiguous() or vs.stride(1) != 1 or vs.shape[1] < 16:
        raise ValueError("layernorm_bwd_lora: contiguous up, row-major vs with 16 columns")
    dx = torch.empty(M, D, dtype=BF16, device=x.device)
    call("vpt_layernorm_bwd_lora", dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), mean.data_ptr(),
         rstd.data_ptr(), w.data_ptr(), _p(dres), 0 if dres is None else dres.stride(0), dx.data_ptr(), dx.stride(0),
         M, D, up.data_ptr(), vs.data_ptr(), vs.stride(0), float(alpha), stream())
    return dx


def layernorm_bwd_blocks(M: int) -> int:
    return _lib.lib.vpt_layernorm_bwd_blocks(M)


def geglu_fwd(x12, out=None):
    M, F2 = x12.shape
    out = torch.empty(M, F2 // 2, dtype=BF16, device=x12.device) if out is None else out
    call("vpt_geglu_fwd", x12.data_ptr(), x12.stride(0), F2 // 2, M, out.data_ptr(), stream())
    return out


def geglu_fwd_lora(x12, down, alpha: float, ds, out=None):
    """geglu_fwd and, in the same launch, ds = bf16(alpha * out . down^T) (down [16, F]; csrc/sdxl.hip
    geglu_fwd_lora_kernel). Returns out."""
    M, F2 = x12.shape
    _chk(down, BF16, "down")
    if not (down.is_contiguous() and down.shape == (16, F2 // 2) and ds.stride(1) == 1 and ds.shape[1] >= 16):
        raise ValueError("geglu_fwd_lora: contiguous down [16, F], row-major ds with 16 columns")
    out = torch.empty(M, F2 // 2, dtype=BF16, device=x12.device) if out is None else out
    tk = tickets(x12.device, (M + 15) // 16)
    part = workspace(x12.device, "geglu_lora", int(call("vpt_geglu_lora_partials_bytes", M, F2 // 2)) // 4)
    call("vpt_geglu_fwd_lora", x12.data_ptr(), x12.stride(0), F2 // 2, M, out.data_ptr(), out.stride(0),
         down.data_ptr(), ds.data_ptr(), ds.stride(0), float(alpha), tk.data_ptr(), part.data_ptr(), stream())
    return out


def geglu_bwd(dy, x12, dx12=None):
    M, F2 = x12.shape
    dx12 = torch.empty_like(x12) if dx12 is None else dx12
    call("vpt_geglu_bwd", dy.data_ptr(), x12.data_ptr(), x12.stride(0), F2 // 2, M, dx12.data_ptr(), dx12.stride(0),
         stream())
    return dx12


def geglu_bwd_lora(dy, x12, up, alpha: float, vs, dx12=None):
    """geglu_bwd and, in the same launch, vs = bf16(alpha * dx12 . up) (up [2F, 16]; csrc/sdxl.hip
    geglu_bwd_lora_kernel). Returns dx12."""
    M, F2 = x12.shape
    _chk(up, BF16, "up")
    if not (dy.is_contiguous() and up.is_contiguous() and up.shape == (F2, 16) and vs.stride(1) == 1
            and vs.shape[1] >= 16):
        raise ValueError("geglu_bwd_lora: dense dy [M, F], contiguous up [2F, 16], row-major vs with 16 columns")
    dx12 = torch.empty_like(x12) if dx12 is None else dx12
    tk = tickets(x12.device, (M + 15) // 16)
    part = workspace(x12.device, "geglu_lora", int(call("vpt_geglu_lora_partials_bytes", M, F2 // 2)) // 4)
    call("vpt_geglu_bwd_lora", dy.data_ptr(), x12.data_ptr(), x12.stride(0), F2 // 2, M, dx12.data_ptr(),
         dx12.stride(0), up.data_ptr(), vs.data_ptr(), vs.stride(0), float(alpha), tk.data_ptr(), part.data_ptr(),
         stream())
    return dx12


def groupnorm_fwd(x, w, b, B, C, G, HW, out=None, mean=None, rstd=None, eps=1e-6):
    """x NCHW bf16 [B, C, HW] -> GroupNorm(G, C) output NCHW bf16; mean / rstd [B*G] f32 (for the backward)."""
    out = torch.empty_like(x) if out is None else out
    mean = torch.empty(B * G, dtype=F32, device=x.device) if mean is None else mean
    rstd = torch.empty(B * G, dtype=F32, device=x.device) if rstd is None else rstd
    call("vpt_groupnorm_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), mean.data_ptr(),
         rstd.data_ptr(), B, C, G, HW, eps, stream())
    return out, mean, rstd


def groupnorm_bwd(dy, x, mean, rstd, w, B, C, G, HW, dres=None, dx=None):
    dx = torch.empty_like(x) if dx is None else dx
    call("vpt_groupnorm_bwd", dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), w.data_ptr(), _p(dres),
         dx.data_ptr(), B, C, G, HW, stream())
    return dx


def transpose_add(src, B, R, S, add=None, out=None):
    """out[b][s][r] = src[b][r][s] (+ add[b][s][r]) for bf16 src [B, R, S] (R, S multiples of 8)."""
    out = torch.empty(B, S, R, dtype=BF16, device=src.device) if out is None else out
    call("vpt_transpose_add", src.data_ptr(), _p(add), out.data_ptr(), B, R, S, stream())
    return out


# ----------------------------------------------------------------------------- SDXL flow matching
def flow_noise(x, t, B, z, eps=None, eps_in=None, noise_scale=1.0, clean_at_zero=False, seed=0):
    """prepare_scaled_noised_latents (src/modules/loss/flow_match.py:60-74) on bf16 latents x [B, ...]:
    eps = bf16(randn * noise_scale) (counter RNG, or eps_in), z = t x + (1 - t) eps (bf16)."""
    n = x.numel() // B
    call("vpt_flow_noise", x.data_ptr(), t.data_ptr(), n, B, float(noise_scale), int(clean_at_zero), int(seed),
         _p(eps_in), z.data_ptr(), _p(eps), stream())
    return z


_LOSS_PART: dict = {}


def velocity_loss(v, x, eps, loss, dv=None):
    """loss_with_predicted_velocity (flow_match.py:85-96): loss (f32 [1]) = mean((v - (eps - x))^2),
    dv = d loss / d v (bf16); deterministic block sums."""
    nb = int(call("vpt_velocity_loss_blocks"))
    part = _LOSS_PART.get(v.device)
    if part is None:
        part = _LOSS_PART[v.device] = torch.empty(nb, dtype=F32, device=v.device)
    _launch("velocity_loss", v.numel() * (6 + (2 if dv is not None else 0)),
            lambda: call("vpt_velocity_loss", v.data_ptr(), x.data_ptr(), eps.data_ptr(), v.numel(), _p(dv),
                         part.data_ptr(), loss.data_ptr(), stream()))
    return loss


def sinusoid_embed(vals, dim, out=None):
    """get_timestep_embedding(vals, dim, flip_sin_to_cos=True, downscale_freq_shift=0) -> bf16 [R, dim]."""
    R = vals.numel()
    out = torch.empty(R, dim, dtype=BF16, device=vals.device) if out is None else out
    call("vpt_sinusoid_embed", vals.data_ptr(), R, dim, out.data_ptr(), stream())
    return out


def space_to_depth(src, B, C, H, W, r, out=None, inverse=False):
    """NCHW [B,C,H,W] -> tokens [B, (H/r)(W/r), C r r] (pixel_unshuffle + permute); inverse: tokens -> NCHW."""
    if out is None:
        out = torch.empty((B, C, H, W) if inverse else (B, (H // r) * (W // r), C * r * r), dtype=BF16,
                          device=src.device)
    call("vpt_space_to_depth", src.data_ptr(), out.data_ptr(), B, C, H, W, r, int(inverse), stream())
    return out


def add_bf16(a, b, out=None):
    out = torch.empty_like(a) if out is None else out
    call("vpt_add_bf16", a.data_ptr(), b.data_ptr(), a.numel(), out.data_ptr(), stream())
    return out


def scale_bf16_2d(a, s, out=None):
    """s * a on a row-strided 2-D view (in place when out is a)."""
    out = torch.empty_like(a) if out is None else out
    call("vpt_scale_bf16_2d", a.data_ptr(), a.stride(0), a.shape[0], a.shape[1], float(s), out.data_ptr(), out.stride(0),
         stream())
    return out


def scale_bf16(a, s, out=None):
    out = torch.empty_like(a) if out is None else out
    call("vpt_scale_bf16", a.data_ptr(), a.numel(), float(s), out.data_ptr(), stream())
    return out


def nf4_dequant(packed, qabsmax, absmax2, code2, offset, n, out):
    def run():
        call("vpt_nf4_dequant", packed.data_ptr(), qabsmax.data_ptr(), absmax2.data_ptr(), code2.data_ptr(),
             offset.data_ptr(), n, out.data_ptr(), stream())
    _launch("nf4_dequant", 2.5 * n, run)  # algorithmic HBM bytes: 0.5 B of codes in, 2 B of bf16 out per weight
    return out


class _Nf4Job(ctypes.Structure):
    """VptNf4Job (include/vpt_hip.h)."""
    _fields_ = [("packed", ctypes.c_void_p), ("qabsmax", ctypes.c_void_p), ("absmax2", ctypes.c_void_p),
                ("code2", ctypes.c_void_p), ("offset", ctypes.c_void_p), ("out", ctypes.c_void_p), ("n", ctypes.c_long)]


def nf4_dequant_batch(pairs):
    """[(NF4Weight, bf16 out)] -> one vpt_nf4_dequant_batch launch per 16 tensors."""
    for i in range(0, len(pairs), 16):
        chunk = pairs[i:i + 16]
        jobs = (_Nf4Job * len(chunk))(*[_Nf4Job(w.packed.data_ptr(), w.qabsmax.data_ptr(), w.absmax2.data_ptr(),
                                                 w.code2.data_ptr(), w.offset.data_ptr(), out.data_ptr(), w.numel)
                                         for w, out in chunk])
        _launch("nf4_dequant", 2.5 * sum(w.numel for w, _ in chunk),
                lambda: call("vpt_nf4_dequant_batch", ctypes.cast(jobs, ctypes.c_void_p), len(chunk), stream()))
    return [out for _, out in pairs]


def gemm_nf4(a, w, forward: bool, out, *, lora_a=None, lora_b=None, bias=None, resid=None, out_mode=OUT_BF16,
             alpha=1.0):
    """NF4 dequant-in-GEMM (csrc/gemm.hip gemm_nf4_kernel). `w` is a vpt.sdxl.NF4Weight [N_w, K_w].
    forward: out[M, N_w] = a[M, K_w] . Wd^T (+bias) (+ lora_a[M, r] . lora_b[N_w, r]^T)
    dgrad:   out[M, K_w] = a[M, N_w] . Wd      (+ lora_a[M, r] . lora_b[r, K_w])"""
    _chk(a, BF16, "a")
    _chk(out, BF16 if out_mode == OUT_BF16 else F32, "out")
    M = a.shape[0]
    Nw, Kw = w.shape
    N, K = (Nw, Kw) if forward else (Kw, Nw)
    if a.shape[1] != K or out.shape[0] != M or out.shape[1] != N:
        raise ValueError(f"gemm_nf4: a {tuple(a.shape)} / out {tuple(out.shape)} do not match W {w.shape}")
    r = 0
    if lora_a is not None:
        _chk(lora_a, BF16, "lora_a")
        _chk(lora_b, BF16, "lora_b")
        r = lora_a.shape[1]
        if tuple(lora_b.shape) != ((N, r) if forward else (r, N)):
            raise ValueError("gemm_nf4: lora_b shape")

    def run():
        call("vpt_gemm_nf4", a.data_ptr(), a.stride(0), w.packed.data_ptr(), w.qabsmax.data_ptr(),
             w.absmax2.data_ptr(), w.code2.data_ptr(), w.offset.data_ptr(), Kw, int(forward), _p(lora_a),
             0 if lora_a is None else lora_a.stride(0), _p(lora_b), 0 if lora_b is None else lora_b.stride(0), r,
             out.data_ptr(), out.stride(0), M, N, K, _p(bias), _p(resid), 0 if resid is None else resid.stride(0),
             out_mode, float(alpha), stream())
    pr = PROBES.get("gemm_nf4")
    if pr is None:
        run()
    else:
        pr.record(2.0 * M * N * (K + r), run, key=f"{'fwd' if forward else 'dgrad'} M{M} N{N} K{K}")
    return out


def lora_proj_grouped(x, x_goff: int, w, w_goff: int, G: int, w_kmajor: bool, out, alpha=1.0):
    """out[:, 16g:16g+16] = alpha * X_g . W_g^T for g < G in one launch, X_g = the [M, K] view at x + g * x_goff and
    W_g = the down [16, K] / up [K, 16] at w + g * w_goff (element offsets; csrc/gemm.hip lora_proj, grouped)."""
    _chk(x, BF16, "x")
    _chk(w, BF16, "w")
    M = x.shape[0]
    K = w.shape[1] if w_kmajor else w.shape[0]
    if x.stride(1) != 1 or out.stride(1) != 1 or out.shape[1] < 16 * G:
        raise ValueError("lora_proj_grouped: row-major x / out with 16 G output columns")
    call("vpt_lora_proj_grouped", x.data_ptr(), x.stride(0), int(x_goff), w.data_ptr(), int(w_kmajor), int(w_goff),
         out.data_ptr(), out.stride(0), M, K, 16, G, float(alpha), stream())
    return out


def lora_proj(x, w, w_kmajor: bool, out, alpha=1.0):
    """out[M, 16] = alpha * x[M, K] . W^T, W = down [16, K] (w_kmajor) or up [K, 16] (csrc/gemm.hip lora_proj)."""
    _chk(x, BF16, "x")
    _chk(w, BF16, "w")
    M, K = x.shape
    call("vpt_lora_proj", x.data_ptr(), x.stride(0), w.data_ptr(), int(w_kmajor), out.data_ptr(), out.stride(0), M, K,
         16, float(alpha), stream())
    return out


_LORA_WS: dict = {}  # per (device, tag, bytes): split slabs, reused across launches on one stream


def _lora_ws(dev, tag, nbytes):
    ws = _LORA_WS.get((dev, tag, nbytes))
    if ws is None:
        ws = _LORA_WS[(dev, tag, nbytes)] = torch.empty(nbytes // 4, dtype=F32, device=dev)
    return ws


class _LoraReduceJob(ctypes.Structure):
    """VptLoraReduceJob (include/vpt_hip.h)."""
    _fields_ = [("part", ctypes.c_void_p), ("g", ctypes.c_void_p), ("n", ctypes.c_int), ("splits", ctypes.c_int),
                ("trans", ctypes.c_int), ("reserved", ctypes.c_int)]


class _LoraWgradJob(ctypes.Structure):
    """VptLoraWgradJob (include/vpt_hip.h)."""
    _fields_ = [("X", ctypes.c_void_p), ("ldx", ctypes.c_long), ("S", ctypes.c_void_p), ("lds", ctypes.c_long),
                ("part", ctypes.c_void_p), ("N", ctypes.c_int), ("M", ctypes.c_int)]


class _LoraBatch:
    """Adapter gradients collected by lora_wgrad_batch(): the slab products of every target deferred to the end of
    the block and launched as one grid (vpt_lora_wgrad_partial_batch, up to 24 one-sided jobs), then one
    vpt_lora_wgrad_reduce_batch launch per 32 jobs (2 per LoRA target) -- instead of two launches per target.
    The operand tensors are held until the flush (their memory is not reused before the slab launch)."""

    def __init__(self, side=None):
        self.jobs: list = []
        self.pjobs: list = []  # deferred slab jobs
        self.keep: list = []   # their operand tensors
        self.key = None  # (alpha, accumulate) of the pending jobs
        self.nws = 0     # workspaces handed out since the last flush
        self.side = side  # a stream the flushes run on (beside the caller's), or None

    def reserve(self, key, njobs):
        """Called BEFORE a target takes its workspaces: flushes first when its jobs would not fit, so the
        workspace names handed out after a flush never alias slabs that pending jobs still have to reduce."""
        if self.jobs and (key != self.key or len(self.jobs) + njobs > 32):
            self.flush()
        self.key = key

    def ws(self, dev, nbytes):
        self.nws += 1
        return _lora_ws(dev, f"batch{self.nws}", nbytes)

    def add(self, jobs):
        assert len(self.jobs) + len(jobs) <= 32
        self.jobs.extend(jobs)

    def defer(self, pjobs, tensors):
        self.pjobs.extend(pjobs)
        self.keep.extend(tensors)

    def flush(self):
        if not self.pjobs and not self.jobs:
            return
        ctx = contextlib.nullcontext()
        if self.side is not None:
            # the slab and reduce launches on the side stream, behind everything the caller's stream enqueued
            # (the operands); the operand tensors are marked as used there so the allocator does not hand their
            # memory out again before these launches ran; the workspaces are touched by the side stream alone
            self.side.wait_stream(torch.cuda.current_stream())
            for t in self.keep:
                t.record_stream(self.side)
            ctx = torch.cuda.stream(self.side)
        with ctx:
            for i in range(0, len(self.pjobs), 24):
                chunk = self.pjobs[i:i + 24]
                arr = (_LoraWgradJob * len(chunk))(*chunk)
                call("vpt_lora_wgrad_partial_batch", ctypes.addressof(arr), len(chunk), stream())
            if self.jobs:
                arr = (_LoraReduceJob * len(self.jobs))(*self.jobs)
                call("vpt_lora_wgrad_reduce_batch", ctypes.addressof(arr), len(self.jobs), float(self.key[0]),
                     int(self.key[1]), stream())
        self.pjobs, self.keep = [], []
        self.jobs, self.nws = [], 0


_LORA_BATCH: _LoraBatch | None = None
# False = each target's slab launch at its call (round-2 behaviour); default: deferred to the block's end.
# Module attributes, not environment switches: tools/ A/B scripts assign them in-process.
_LORA_DEFER = True
_LORA_BATCHED = True


@contextlib.contextmanager
def lora_wgrad_batch(side=None):
    """Within the block, lora_wgrad2 only writes its split-M slabs (each target into its own workspace) and the
    reduces run batched at exit (or every 32 jobs): same results, ~1/16 of the reduce launches. side: a stream the
    batched launches run on beside the caller's (the caller joins it before reading the adapter gradients)."""
    global _LORA_BATCH
    if not _LORA_BATCHED:  # per-target reduces (A/B: tools/c5_knob_ab.py)
        yield
        return
    outer = _LORA_BATCH
    _LORA_BATCH = _LoraBatch(side)
    try:
        yield
        _LORA_BATCH.flush()
    finally:
        _LORA_BATCH = outer


def lora_wgrad2(dy, ds, g_up, x, vs, g_down, accumulate=True, alpha=1.0):
    """Both LoRA adapter gradients (csrc/gemm.hip lora_wgrad): g_up[N_out,16] (+)= alpha dy^T ds and
    g_down[16,N_in] (+)= alpha vs^T x, f32, deterministic split-M partial sums; 2 launches (the reduce batched
    with other targets' inside lora_wgrad_batch())."""
    M, n_out = dy.shape
    n_in = x.shape[1]
    b = _LORA_BATCH
    if b is None:
        ws_up = _lora_ws(dy.device, "up", int(_lib.lib.vpt_lora_wgrad_workspace(M, n_out)))
        ws_dn = _lora_ws(dy.device, "down", int(_lib.lib.vpt_lora_wgrad_workspace(M, n_in)))
        call("vpt_lora_wgrad2", dy.data_ptr(), dy.stride(0), ds.data_ptr(), ds.stride(0), g_up.data_ptr(), n_out,
             x.data_ptr(), x.stride(0), vs.data_ptr(), vs.stride(0), g_down.data_ptr(), n_in, M, int(accumulate),
             float(alpha), ws_up.data_ptr(), ws_dn.data_ptr(), stream())
        return
    for t, dt in ((g_up, F32), (g_down, F32)):
        _chk(t, dt, "adapter grad")
    b.reserve((float(alpha), int(accumulate)), 2)
    ws_up = b.ws(dy.device, int(_lib.lib.vpt_lora_wgrad_workspace(M, n_out)))
    ws_dn = b.ws(dy.device, int(_lib.lib.vpt_lora_wgrad_workspace(M, n_in)))
    if _LORA_DEFER:
        for t in (dy, ds, x, vs):
            if t.stride(1) != 1 or t.stride(0) % 8:
                raise ValueError("lora_wgrad2: row-major operands with 16-B leading dims")
        b.defer([_LoraWgradJob(dy.data_ptr(), dy.stride(0), ds.data_ptr(), ds.stride(0), ws_up.data_ptr(), n_out, M),
                 _LoraWgradJob(x.data_ptr(), x.stride(0), vs.data_ptr(), vs.stride(0), ws_dn.data_ptr(), n_in, M)],
                (dy, ds, x, vs))
    else:
        if b.side is not None:  # the slabs may still be read by a side-stream reduce of an earlier flush
            torch.cuda.current_stream().wait_stream(b.side)
        call("vpt_lora_wgrad2_partial", dy.data_ptr(), dy.stride(0), ds.data_ptr(), ds.stride(0), n_out,
             x.data_ptr(), x.stride(0), vs.data_ptr(), vs.stride(0), n_in, M, ws_up.data_ptr(), ws_dn.data_ptr(),
             stream())
    b.add([_LoraReduceJob(ws_up.data_ptr(), g_up.data_ptr(), n_out, call("vpt_lora_wgrad_splits", M, n_out), 0, 0),
           _LoraReduceJob(ws_dn.data_ptr(), g_down.data_ptr(), n_in, call("vpt_lora_wgrad_splits", M, n_in), 1, 0)])


def nf4_quantize(w, code2, packed, qabsmax, absmax2, offset, scratch):
    call("vpt_nf4_quantize", w.data_ptr(), w.numel(), code2.data_ptr(), packed.data_ptr(), qabsmax.data_ptr(),
         absmax2.data_ptr(), offset.data_ptr(), scratch.data_ptr(), stream())



# ----------------------------------------------------------------------------- bucketed batch preparation
def cover_resize_crop_workspace(in_h, in_w, scaled_h, scaled_w, top, out_h, out_w) -> int:
    return int(call("vpt_cover_resize_crop_workspace", in_h, in_w, scaled_h, scaled_w, top, out_h, out_w))


def cover_resize_crop(img_u8, in_h, in_w, scaled_h, scaled_w, top, left, out_h, out_w, workspace, out):
    """uint8 [in_h, in_w, 3] -> fp16 [3, out_h, out_w] (see include/vpt_hip.h)."""
    if img_u8.dtype != torch.uint8 or not img_u8.is_contiguous():
        raise ValueError("img must be a contiguous uint8 [H, W, 3] GPU tensor")
    if out.dtype != torch.float16 or not out.is_contiguous():
        raise ValueError("out must be a contiguous fp16 [3, h, w] GPU tensor")
    call("vpt_cover_resize_crop", img_u8.data_ptr(), in_h, in_w, scaled_h, scaled_w, top, left, out_h, out_w,
         workspace.data_ptr(), out.data_ptr(), stream())
    return out
