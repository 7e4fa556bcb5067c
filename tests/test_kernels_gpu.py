"""Per-kernel numerics of libvpt_hip.so on the GPU against plain PyTorch fp32 references of the
same op (computed on the same bf16 inputs). Tolerances are stated per test."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vpt import ops as _ops
    return _ops


def rnd(*shape, scale=1.0, dtype=torch.bfloat16, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype).to(DEV)


# ------------------------------------------------------------------------------------ row sums / row copies
@pytest.mark.parametrize("R,C", [(1, 8), (7, 130), (255, 768), (256, 768), (512, 768), (1024, 128), (3168, 128),
                                 (300, 66)])
def test_reduce_rows(ops, R, C):
    """out (=|+=) the column sums of an f32 [R, C] partial set: within f32 summation error of a float64 sum,
    and bitwise reproducible (fixed summation order)."""
    part = rnd(R, C, dtype=torch.float32, seed=R + C)
    out = torch.empty(C, device=DEV)
    ops.reduce_rows(part, out)
    ref = part.double().sum(0)
    assert (out.double() - ref).abs().max().item() < 1e-5 * (part.abs().sum(0).max().item() + 1)
    again = torch.empty(C, device=DEV)
    ops.reduce_rows(part, again)
    assert torch.equal(out, again)
    base = rnd(C, dtype=torch.float32, seed=5)
    acc = base.clone()
    ops.reduce_rows(part, acc, accumulate=True)
    assert (acc.double() - (base.double() + ref)).abs().max().item() < 1e-5 * (part.abs().sum(0).max().item() + 2)


@pytest.mark.parametrize("B,rows,row0,cnt,D", [(2, 300, 0, 256, 64), (3, 97, 5, 80, 136), (1, 16, 0, 16, 8)])
def test_copy_rows_scatter_zero_rest(ops, B, rows, row0, cnt, D):
    """copy_rows reverse with zero_rest: the slice's rows from dense, every other row zero (no prior fill)."""
    dense = rnd(B * cnt, D, seed=11)
    seq = torch.full((B * rows, D), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops.copy_rows(seq, rows, row0, cnt, dense, B, reverse=True, zero_rest=True)
    ref = torch.zeros(B, rows, D, dtype=torch.bfloat16, device=DEV)
    ref[:, row0:row0 + cnt] = dense.view(B, cnt, D)
    assert torch.equal(seq.view(B, rows, D), ref)
    back = torch.empty_like(dense)
    ops.copy_rows(seq, rows, row0, cnt, back, B)
    assert torch.equal(back, dense)


# ------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 136, 200), (1000, 768, 768), (64, 2304, 768)])
def test_gemm_forward(ops, M, N, K):
    x = rnd(M, K, seed=1)
    w = rnd(N, K, scale=0.05, seed=2)
    b = rnd(N, scale=0.1, seed=3)
    y = ops.linear(x, w, bias=b)
    ref = x.float() @ w.float().t() + b.float()
    assert rel(y, ref) < 5e-3  # bf16 output rounding


def test_gemm_identity_asymmetric(ops):
    # A = I with an asymmetric B catches a transposed C write (guide §3).
    n = 128
    eye = torch.eye(n, dtype=torch.bfloat16, device=DEV)
    b = (torch.arange(n * n, dtype=torch.float32, device=DEV).view(n, n) % 61 - 30).to(torch.bfloat16)
    y = ops.linear(eye, b)  # eye @ b.T = b.T
    assert torch.equal(y.float(), b.float().t())


def test_gemm_residual_silu(ops):
    M, N, K = 384, 256, 256
    x, w, b, r = rnd(M, K, seed=4), rnd(N, K, scale=0.05, seed=5), rnd(N, scale=0.1, seed=6), rnd(M, N, seed=7)
    y = ops.linear(x, w, bias=b, resid=r)
    lin = (x.float() @ w.float().t() + b.float()).to(torch.bfloat16)
    ref = (lin.float() + r.float()).to(torch.bfloat16)
    assert rel(y, ref) < 5e-3
    ys = ops.linear(x, w, bias=b, act=ops.ACT_SILU)
    refs = torch.nn.functional.silu(x.float() @ w.float().t() + b.float())
    assert rel(ys, refs) < 5e-3


@pytest.mark.parametrize("M,N,K", [(512, 256, 384), (1000, 768, 200)])
def test_gemm_dgrad(ops, M, N, K):
    dy = rnd(M, N, seed=8)
    w = rnd(N, K, scale=0.05, seed=9)
    dx = ops.linear_dgrad(dy, w)
    assert rel(dx, dy.float() @ w.float()) < 5e-3


@pytest.mark.parametrize("M,N,K,splits", [(1000, 256, 128, 1), (4170, 768, 768, 4), (333, 136, 64, 2)])
def test_gemm_wgrad(ops, M, N, K, splits):
    dy = rnd(M, N, seed=10)
    x = rnd(M, K, seed=11)
    out = torch.zeros(N, K, dtype=torch.float32, device=DEV)
    ops.linear_wgrad(dy, x, out, splits=splits)
    ref = dy.float().t() @ x.float()
    assert rel(out, ref) < 1e-5
    ops.linear_wgrad(dy, x, out, accumulate=True)
    assert rel(out, 2 * ref) < 1e-5


@pytest.mark.parametrize("geo", [128, 256])
@pytest.mark.parametrize("M,N,K", [(700, 264, 200), (300, 512, 136), (2100, 768, 768), (520, 264, 40),
                                   (512, 512, 32), (776, 1032, 96)])
def test_gemm_geometries_all_directions(ops, geo, M, N, K):
    """Both production tile geometries (128 = T128, 256 = the BK=32 ping-pong ring), forced per call
    (vpt_gemm_bf16_tiled), all three GEMM directions, ragged M/N, partial K tiles (K % 32 != 0
    exercises the clamped-DMA + LDS zeroing path for k-major and mn-major tiles) and ring depths 1-3
    (K = 32, 96)."""
    x = rnd(M, K, seed=80)
    w = rnd(N, K, scale=0.05, seed=81)
    b = rnd(N, scale=0.1, seed=82)
    dy = rnd(M, N, seed=83)
    assert rel(ops.linear(x, w, bias=b, geometry=geo), x.float() @ w.float().t() + b.float()) < 5e-3
    assert rel(ops.linear_dgrad(dy, w, geometry=geo), dy.float() @ w.float()) < 5e-3
    out = torch.empty(N, K, dtype=torch.float32, device=DEV)
    for splits in (1, 3):
        ops.linear_wgrad(dy, x, out, splits=splits, geometry=geo)
        assert rel(out, dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("grid", [1, 3, 8, 37])
def test_gemm_ring_persistent_grid(ops, grid):
    """The persistent 256x256 ring kernel with fewer blocks than work items: every block walks several
    (tile, split-K slice) items (epilogue -> next item's DMA in one block), all three directions."""
    M, N, K = 1100, 776, 200
    t = dict(geometry=256, ring_grid=grid)
    x = rnd(M, K, seed=90)
    w = rnd(N, K, scale=0.05, seed=91)
    b = rnd(N, scale=0.1, seed=92)
    dy = rnd(M, N, seed=93)
    assert rel(ops.linear(x, w, bias=b, **t), x.float() @ w.float().t() + b.float()) < 5e-3
    assert rel(ops.linear_dgrad(dy, w, **t), dy.float() @ w.float()) < 5e-3
    out = torch.empty(N, K, dtype=torch.float32, device=DEV)
    for splits in (1, 5):
        ops.linear_wgrad(dy, x, out, splits=splits, **t)
        assert rel(out, dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("grid", [3, 0])
@pytest.mark.parametrize("M,N,K", [(1100, 776, 200), (2100, 768, 768)])
def test_gemm_ring_epilogue_loads(ops, grid, M, N, K):
    """Ring epilogue modes that read memory (residual add, f32 accumulate into C), whose operands are
    preloaded in groups before the next item's LDS-DMA: several items per block (grid 3) and one block
    per CU (grid 0), ragged last row / column tiles. Against the T128 kernel (same roundings) and fp32."""
    t = dict(geometry=256, ring_grid=grid)
    x = rnd(M, K, seed=140)
    w = rnd(N, K, scale=0.05, seed=141)
    b = rnd(N, scale=0.1, seed=142)
    r = rnd(M, N, seed=143)
    y = ops.linear(x, w, bias=b, resid=r, **t)
    lin = (x.float() @ w.float().t() + b.float()).to(torch.bfloat16)
    assert rel(y, (lin.float() + r.float()).to(torch.bfloat16)) < 5e-3
    y128 = ops.linear(x, w, bias=b, resid=r, geometry=128)
    assert (y.float() - y128.float()).abs().max().item() <= 2 * (y128.float().abs().max().item() * 2 ** -8)
    dy = rnd(M, N, seed=144)
    out0 = rnd(N, K, seed=145, dtype=torch.float32)
    out = out0.clone()
    ops.linear_wgrad(dy, x, out, accumulate=True, splits=1, **t)
    assert rel(out, out0 + dy.float().t() @ x.float()) < 1e-5


@pytest.mark.parametrize("geo,grid,splits", [(256, 0, 1), (256, 3, 5), (256, 0, 9), (128, 0, 1), (128, 0, 3)])
@pytest.mark.parametrize("M,N,K", [(1100, 776, 200), (4170, 768, 768), (333, 264, 136)])
def test_linear_wgrad_fused_bias(ops, geo, grid, splits, M, N, K):
    """Weight + bias gradient in one call (vpt_linear_wgrad): on the ring the bias sums are MFMAs of the dy
    fragments against an all-ones fragment in the first output tile's items (ragged row tiles, several
    items per block, split-K partial sums reduced with the slabs); on T128 the colsum fallback. Store and
    accumulate modes, against fp32 torch and against the standalone colsum kernel."""
    dy = rnd(M, N, seed=150)
    x = rnd(M, K, seed=151)
    out = torch.empty(N, K, dtype=torch.float32, device=DEV)
    b = torch.empty(N, dtype=torch.float32, device=DEV)
    ops.linear_wgrad(dy, x, out, splits=splits, bias_out=b, geometry=geo, ring_grid=grid)
    ref_w, ref_b = dy.float().t() @ x.float(), dy.float().sum(0)
    assert rel(out, ref_w) < 1e-5
    assert rel(b, ref_b) < 1e-5
    bc = torch.empty_like(b)
    ops.bias_grad(dy, bc)
    assert rel(b, bc) < 1e-6
    ops.linear_wgrad(dy, x, out, accumulate=True, splits=splits, bias_out=b, geometry=geo, ring_grid=grid)
    assert rel(out, 2 * ref_w) < 1e-5
    assert rel(b, 2 * ref_b) < 1e-5


@pytest.mark.parametrize("geo,splits,bias", [(256, 1, True), (256, 4, True), (256, 3, False), (128, 1, False),
                                             (128, 2, True), (0, 1, False)])
def test_linear_wgrad_rows_sum_job(ops, geo, splits, bias):
    """vpt_linear_wgrad_rr: the weight / bias gradients bitwise what vpt_linear_wgrad gives, and the riding column sum
    (store and accumulate) within f32 summation error of a float64 sum, bitwise reproducible -- also where no split-K
    reduce launch would otherwise run (splits 1, no ring bias sums)."""
    M, N, K = 2100, 768, 512
    dy = rnd(M, N, seed=160)
    x = rnd(M, K, seed=161)
    part = rnd(512, 768, dtype=torch.float32, seed=162)
    w1, w2 = (torch.empty(N, K, dtype=torch.float32, device=DEV) for _ in range(2))
    b1, b2 = (torch.empty(N, dtype=torch.float32, device=DEV) for _ in range(2))
    r1, r2 = torch.empty(768, device=DEV), torch.empty(768, device=DEV)
    ops.linear_wgrad(dy, x, w1, splits=splits, bias_out=b1 if bias else None, geometry=geo)
    ops.linear_wgrad(dy, x, w2, splits=splits, bias_out=b2 if bias else None, geometry=geo, rows_sum=(part, r1, False))
    assert torch.equal(w1, w2)
    if bias:
        assert torch.equal(b1, b2)
    ref = part.double().sum(0)
    tol = 1e-5 * part.abs().sum(0).max().item()
    assert (r1.double() - ref).abs().max().item() < tol
    ops.linear_wgrad(dy, x, w2, splits=splits, geometry=geo, rows_sum=(part, r2, False))
    assert torch.equal(r1, r2)
    base = r1.clone()
    ops.linear_wgrad(dy, x, w2, splits=splits, geometry=geo, rows_sum=(part, r1, True))
    assert (r1.double() - (base.double() + ref)).abs().max().item() < 2 * tol


@pytest.mark.parametrize("M", [5192, 33360])
def test_swiglu_fused_epilogues_match_unfused(ops, M):
    """The fused SwiGLU ring epilogues the bench runs (forward sw=1: W1|W2 GEMM -> x12, h; backward sw=2:
    W3 dgrad -> dx12 with dh kept in registers) against the unfused GEMM + elementwise kernels on the same
    inputs. M = 5192 is the smallest fused shape here (21 x 8 >= 160 tiles) with a partial last 256-row
    tile; M = 33360 is the bench's B = 8 x 1024^2 token count. Both paths run the same ring GEMM on the
    same operands, so the results are bit-identical."""
    D, F = 768, 2048
    assert (M + 255) // 256 * (F // 256) >= 160  # the fused path is taken (swiglu_ring_ok)
    x = rnd(M, D, seed=130)
    w12 = rnd(2 * F, D, scale=0.03, seed=131)
    b12 = rnd(2 * F, scale=0.1, seed=132)
    x12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=DEV)
    h = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    ops.linear_swiglu(x, w12, b12, x12, h)
    x12_u = ops.linear(x, w12, bias=b12)
    h_u = torch.empty_like(h)
    ops.swiglu_fwd(x12_u, h_u)
    assert torch.equal(x12, x12_u)
    assert torch.equal(h, h_u)
    x12f = x12.float()
    # torch's bf16 silu (libm expf + IEEE division in f32) vs the kernels' v_exp_f32 + v_rcp_f32 sigmoid: at
    # most one bf16 ulp apart (csrc/common.h sigmoid_hw), and equal almost everywhere
    h_ref = (torch.nn.functional.silu(x12f[:, :F]).bfloat16().float() * x12f[:, F:]).bfloat16()
    assert ((h.float() - h_ref.float()).abs() <= h_ref.float().abs() * 2 ** -7 + 1e-30).all()
    assert (h != h_ref).float().mean().item() < 0.02
    # backward
    dy = rnd(M, D, seed=133)
    w3 = rnd(D, F, scale=0.03, seed=134)
    dx12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=DEV)
    ops.linear_dgrad_swiglu(dy, w3, x12, dx12)
    dh = ops.linear_dgrad(dy, w3)
    dx12_u = torch.empty_like(dx12)
    ops.swiglu_bwd(dh, x12, dx12_u)
    assert torch.equal(dx12, dx12_u)
    # and against torch autograd of the reference's bf16 SwiGLU graph (denoiser.py:480-506)
    a = x12[:, :F].clone().requires_grad_(True)
    b = x12[:, F:].clone().requires_grad_(True)
    (torch.nn.functional.silu(a) * b).backward(dh)
    assert rel(dx12[:, :F], a.grad) < 1e-2 and rel(dx12[:, F:], b.grad) < 1e-2


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("splits", [1, 2])
def test_gemm_r2_128_equals_t128(ops, ak, bk, splits):
    """Geometry 1281 (128x128 tiles on the R2 ring's 3-stage LDS-DMA pipeline) == geometry 128 (the two-stage 128x128
    kernel): the same 32-deep K chunks in the same order, so equal outputs -- bf16 with bias + residual, f32 and f32
    accumulate, ragged M / N / K, split-K."""
    M, N, K = 1000, 1280, 1216
    a = rnd(M, K, seed=90) if ak else rnd(K, M, seed=90)
    b = rnd(N, K, scale=0.05, seed=91) if bk else rnd(K, N, scale=0.05, seed=91)
    bias, resid = rnd(N, scale=0.1, seed=92), rnd(M, N, seed=93)
    for out_mode, kw in ((ops.OUT_BF16, dict(bias=bias, resid=resid)), (ops.OUT_F32, {}), (ops.OUT_F32_ACC, {}),
                         (ops.OUT_BF16, dict(bias=bias, act=ops.ACT_SILU)), (ops.OUT_BF16, dict(alpha=0.37))):
        if splits > 1 and ("act" in kw or "alpha" in kw):
            continue  # (split-K: no SiLU / alpha epilogue)
        dt = torch.bfloat16 if out_mode == ops.OUT_BF16 else torch.float32
        if out_mode == ops.OUT_F32_ACC:
            if splits > 1:
                continue
            base = rnd(M, N, dtype=torch.float32, seed=94)
            ref, out = base.clone(), base.clone()
        else:
            ref, out = torch.empty(M, N, dtype=dt, device=DEV), torch.full((M, N), float("nan"), dtype=dt, device=DEV)
        ops.gemm(a, ak, b, bk, M, N, K, ref, out_mode=out_mode, splits=splits, geometry=128, **kw)
        ops.gemm(a, ak, b, bk, M, N, K, out, out_mode=out_mode, splits=splits, geometry=1281, **kw)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (out_mode, (out.float() - ref.float()).abs().max().item())


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (37, 136, 96), (130, 264, 40), (257, 1280, 1280), (600, 8, 32)])
@pytest.mark.parametrize("bk", [True, False])
def test_gemm_r2_128_small_and_ragged(ops, M, N, K, bk):
    """Geometry 1281 at tiny and ragged shapes (one row, partial row / column tiles, a partial 32-deep K tile, N = 8)
    == geometry 128, with bias + residual."""
    a = rnd(M, K, seed=100)
    b = rnd(N, K, scale=0.1, seed=101) if bk else rnd(K, N, scale=0.1, seed=101)
    bias, resid = rnd(N, scale=0.1, seed=102), rnd(M, N, seed=103)
    ref = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops.gemm(a, True, b, bk, M, N, K, ref, bias=bias, resid=resid, geometry=128)
    ops.gemm(a, True, b, bk, M, N, K, out, bias=bias, resid=resid, geometry=1281)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()


def test_gemm_split_matches_unsplit(ops):
    M, N, K = 2048, 384, 256
    dy, x = rnd(M, N, seed=12), rnd(M, K, seed=13)
    a = torch.empty(N, K, dtype=torch.float32, device=DEV)
    b = torch.empty_like(a)
    ops.linear_wgrad(dy, x, a, splits=1)
    ops.linear_wgrad(dy, x, b, splits=8)
    assert rel(a, b) < 1e-6


# ------------------------------------------------------------------------------------ norms
def test_rmsnorm_fwd_bwd(ops):
    M, D = 777, 768
    x = rnd(M, D, seed=20)
    w = (1 + rnd(D, scale=0.1, seed=21).float()).to(torch.bfloat16)
    y, rstd = ops.rmsnorm_fwd(x, w)
    xf = x.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    ref = torch.nn.functional.rms_norm(xf, (D,), weight=wf, eps=1e-6)
    assert rel(y, ref) < 5e-3
    assert rel(rstd, torch.rsqrt(x.float().pow(2).mean(-1) + 1e-6)) < 1e-5
    dy = rnd(M, D, seed=22)
    dres = rnd(M, D, seed=23)
    dx, part = ops.rmsnorm_bwd(dy, x, rstd, w, dres=dres)
    dw = torch.zeros(D, device=DEV)
    ops.reduce_rows(part, dw)
    ref.backward(dy.float())
    assert rel(dx, xf.grad + dres.float()) < 5e-3
    assert rel(dw, wf.grad) < 1e-4


def _rope_tables(rows, seed=30):
    g = torch.Generator(device="cpu").manual_seed(seed)
    ang = torch.rand(rows, 32, generator=g) * 6.0
    return torch.cos(ang).to(DEV), torch.sin(ang).to(DEV)


def _ref_qknorm_rope(qkv, wq, wk, cos, sin, rows_per_seq):
    M = qkv.shape[0]
    pos = torch.arange(M, device=DEV) % rows_per_seq
    fc = torch.complex(cos[pos], sin[pos])  # [M,32]
    outs = []
    for i, w in enumerate((wq, wk)):
        x = qkv[:, i * 768:(i + 1) * 768].float().view(M, 12, 64)
        y = torch.nn.functional.rms_norm(x, (64,), weight=w.float(), eps=1e-6)
        yc = torch.view_as_complex(y.reshape(M, 12, 32, 2)) * fc[:, None, :]
        outs.append(torch.view_as_real(yc).reshape(M, 768))
    return torch.cat(outs, 1)


def test_qknorm_rope_fwd_bwd(ops):
    M, rps = 530, 265
    qkv = rnd(M, 2304, seed=31)
    wq = (1 + rnd(64, scale=0.1, seed=32).float()).to(torch.bfloat16)
    wk = (1 + rnd(64, scale=0.1, seed=33).float()).to(torch.bfloat16)
    cos, sin = _rope_tables(rps)
    out = ops.qknorm_rope_fwd(qkv, wq, wk, cos, sin, rps)
    qf = qkv.float().requires_grad_(True)
    wqf = wq.float().requires_grad_(True)
    wkf = wk.float().requires_grad_(True)
    ref = _ref_qknorm_rope(qf, wqf, wkf, cos, sin, rps)
    assert rel(out, ref) < 8e-3
    g = rnd(M, 1536, seed=34)
    dqkv = torch.zeros(M, 2304, dtype=torch.bfloat16, device=DEV)
    part = ops.qknorm_rope_bwd(g, qkv, wq, wk, cos, sin, rps, dqkv)
    dw = torch.zeros(128, device=DEV)
    ops.reduce_rows(part, dw)
    ref.backward(g.float())
    assert rel(dqkv[:, :1536], qf.grad[:, :1536]) < 8e-3
    assert rel(dw[:64], wqf.grad) < 1e-3
    assert rel(dw[64:], wkf.grad) < 1e-3


@pytest.mark.parametrize("M,rps", [(530, 265), (8 * 4170, 4170), (4 * 1034 + 6, 1034)])
def test_linear_qknorm_rope_fused_epilogue(ops, M, rps):
    """vpt_linear_qknorm_rope (q|k|v projection with the per-head QK-RMSNorm + RoPE in the ring GEMM's epilogue) ==
    linear then qknorm_rope_fwd, bitwise (qkv and qk), at a small M, the C3 1024^2 B=8 shape (ring items with q, k and
    v heads, partial last row tile) and a ragged one; and within bf16 of the fp32 reference."""
    D, K = 768, 768
    x = rnd(M, K, seed=61)
    w = rnd(3 * D, K, scale=0.05, seed=62)
    b = rnd(3 * D, scale=0.1, seed=63)
    wq = (1 + rnd(64, scale=0.1, seed=64).float()).to(torch.bfloat16)
    wk = (1 + rnd(64, scale=0.1, seed=65).float()).to(torch.bfloat16)
    cos, sin = _rope_tables(rps, seed=66)
    qs = ops.attn_q_scale(0.125)
    qkv = torch.empty(M, 3 * D, dtype=torch.bfloat16, device=DEV)
    qk = torch.empty(M, 2 * D, dtype=torch.bfloat16, device=DEV)
    ops.linear_qknorm_rope(x, w, b, qkv, qk, wq, wk, cos, sin, rps, q_scale=qs)
    ref_qkv = ops.linear(x, w, b)
    ref_qk = ops.qknorm_rope_fwd(ref_qkv, wq, wk, cos, sin, rps, q_scale=qs)
    torch.cuda.synchronize()
    assert torch.equal(qkv, ref_qkv)
    assert torch.equal(qk, ref_qk)
    if M < 4096:
        f = _ref_qknorm_rope(qkv.float(), wq.float(), wk.float(), cos, sin, rps)
        f[:, :D] *= qs
        assert rel(qk, f) < 8e-3


# ------------------------------------------------------------------------------------ attention
def prescale_q(ops, t, D, scale=0.125):
    """Copy of t whose first D columns (q) carry the attention kernels' pre-scale (include/vpt_hip.h)."""
    t = t.clone()
    t[:, :D] = (t[:, :D].float() * ops.attn_q_scale(scale)).bfloat16()
    return t


def _attn_ref(q, k, v, bias, scale):
    # q,k,v [B,H,N,64] f32; bias [B,N] additive
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) * scale + bias[:, None, None, :]
    p = torch.softmax(s, -1)
    return torch.einsum("bhqk,bhkd->bhqd", p, v)


@pytest.mark.parametrize("n,n_dense,masked", [(200, 150, True), (330, 330, False), (64, 40, True), (1034, 1024, True),
                                              (700, 520, True)])
def test_attention_fwd_bwd(ops, n, n_dense, masked):
    B, H, rows = 2, 3, ((n + 127) // 128) * 128
    D = H * 64
    qkv = rnd(B * rows, 3 * D, seed=40)
    kb = torch.zeros(B, rows, device=DEV)
    if masked:
        kb[:, n_dense + (n - n_dense) // 2:] = float("-inf")
        kb[1, n_dense:] = 0.0  # second sequence: nothing masked
    o = torch.zeros(B * rows, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B, H, rows, device=DEV)
    qkv_s = prescale_q(ops, qkv, D)
    q4 = ops._t4(qkv_s, B, rows, H, 0)
    k4 = ops._t4(qkv_s, B, rows, H, D)
    v4 = ops._t4(qkv_s, B, rows, H, 2 * D)
    o4 = ops._t4(o, B, rows, H, 0)
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense)

    def heads(t, c0):
        return t[:, c0:c0 + D].float().view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3).contiguous()

    qf = heads(qkv, 0).requires_grad_(True)
    kf = heads(qkv, D).requires_grad_(True)
    vf = heads(qkv, 2 * D).requires_grad_(True)
    bias = kb[:, :n].clone()
    bias[:, n_dense:] = kb[:, n_dense:n]
    ref = _attn_ref(qf, kf, vf, bias, 0.125)
    got = o.view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3).float()
    assert rel(got, ref) < 1e-2

    do = rnd(B * rows, D, seed=41)
    dq = torch.zeros(B * rows, D, dtype=torch.bfloat16, device=DEV)
    dk = torch.zeros_like(dq)
    dv = torch.zeros_like(dq)
    delta = torch.zeros(B, H, rows, device=DEV)
    ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb, ops._t4(dq, B, rows, H),
                 ops._t4(dk, B, rows, H), ops._t4(dv, B, rows, H), B, H, rows, n, n_dense)
    dof = do.float().view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3)
    ref.backward(dof)

    def unh(t):
        return t.view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3).float()

    assert rel(unh(dq), qf.grad) < 2e-2
    assert rel(unh(dk), kf.grad) < 2e-2
    assert rel(unh(dv), vf.grad) < 2e-2


@pytest.mark.parametrize("B,H,n,nk,n_dense,masked", [(2, 3, 200, 200, 150, True), (2, 3, 40, 40, 20, True),
                                                     (1, 2, 64, 64, 64, False), (2, 12, 4170, 4170, 4106, True),
                                                     (3, 5, 1034, 1034, 1024, True), (2, 3, 300, 231, 231, False),
                                                     (2, 3, 1000, 77, 38, True)])
def test_attention_bwd_queue_bitwise(ops, B, H, n, nk, n_dense, masked):
    """vpt_attn_bwd_q (resident blocks pulling the dK/dV and dQ items from per-XCD work queues, the next item's first
    tile staged under the current item's last) is bitwise vpt_attn_bwd (one block per item): self- and cross-attention,
    ragged and sub-tile lengths, masks, fewer items than resident blocks (40 rows) and the C3 shape; three launches in a
    row on the same queue words (each launch resets them) and two streams with their own queues at once."""
    D = H * 64
    q = prescale_q(ops, rnd(B * n, D, seed=90), D)
    kv = rnd(B * nk, 2 * D, seed=91)
    kb = torch.zeros(B, nk, device=DEV)
    if masked:
        kb[0, n_dense + (nk - n_dense) // 2:] = float("-inf")
    o = torch.zeros(B * n, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B, H, n, device=DEV)
    q4, k4, v4, o4 = (ops._t4(q, B, n, H, 0), ops._t4(kv, B, nk, H, 0), ops._t4(kv, B, nk, H, D),
                      ops._t4(o, B, n, H, 0))
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, n, n, n_dense, nk=nk)
    do = rnd(B * n, D, seed=92)

    def run(queue):
        dq = torch.full((B * n, D), 7.0, dtype=torch.bfloat16, device=DEV)
        dkv = torch.full((B * nk, 2 * D), 7.0, dtype=torch.bfloat16, device=DEV)
        delta = torch.zeros(B, H, n, device=DEV)
        ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, n, H, 0), lse, delta, kb, ops._t4(dq, B, n, H, 0),
                     ops._t4(dkv, B, nk, H, 0), ops._t4(dkv, B, nk, H, D), B, H, n, n, n_dense, nk=nk, queue=queue)
        return dq, dkv

    ref = run(False)
    for _ in range(3):
        got = run(True)
        torch.cuda.synchronize()
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    assert ops.attn_queue().abs().sum().item() == 0  # left reset
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for st in streams:
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs.append(run(True))
    torch.cuda.synchronize()
    for got in outs:
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])


@pytest.mark.parametrize("n,n_dense,masked", [(200, 150, True), (330, 330, False), (1034, 1024, True), (700, 520, True)])
def test_attention_bwd_fused_qknorm_rope(ops, n, n_dense, masked):
    """vpt_attn_bwd_qknorm (the QK-RMSNorm + RoPE backward fused into the attention backward's dQ / dK stores) vs an
    fp32 autograd reference of rope(rms(x) w) -> SDPA (denoiser.py:307-316, 98-111, attention.py:98-129), and vs the
    unfused pair (vpt_attn_bwd then vpt_qknorm_rope_bwd). Rows past n (pre-context blocks) are left untouched; masked
    keys get exactly zero gradients."""
    B, H, rows = 2, 3, ((n + 127) // 128) * 128
    D = H * 64
    qkv = rnd(B * rows, 3 * D, seed=50)
    wq = (1 + rnd(64, scale=0.1, seed=51).float()).to(torch.bfloat16)
    wk = (1 + rnd(64, scale=0.1, seed=52).float()).to(torch.bfloat16)
    cos, sin = _rope_tables(rows, seed=53)
    kb = torch.zeros(B, rows, device=DEV)
    if masked:
        kb[:, n_dense + (n - n_dense) // 2:] = float("-inf")
        kb[1, n_dense:] = 0.0
    M = B * rows
    # forward: the production pieces (qknorm_rope_fwd with the q pre-scale, then attention)
    qk = ops.qknorm_rope_fwd(qkv[:, :3 * D], wq, wk, cos, sin, rows, q_scale=ops.attn_q_scale(0.125))
    o = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B, H, rows, device=DEV)
    q4, k4, v4 = ops._t4(qk, B, rows, H, 0), ops._t4(qk, B, rows, H, D), ops._t4(qkv, B, rows, H, 2 * D)
    o4 = ops._t4(o, B, rows, H, 0)
    ops.attn_fwd(q4, k4, v4, o4, lse, kb, B, H, rows, n, n_dense)
    do = rnd(M, D, seed=54)
    sentinel = 7.0
    dqkv = torch.full((M, 3 * D), sentinel, dtype=torch.bfloat16, device=DEV)
    nd = ops.attn_bwd_dw_rows(B, H, n)
    part = torch.full((nd, 128), float("nan"), device=DEV)
    delta = torch.zeros(B, H, rows, device=DEV)
    ops.attn_bwd_qknorm(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb, ops._t4(qkv, B, rows, H, 0),
                        ops._t4(qkv, B, rows, H, D), wq, wk, cos, sin, ops._t4(dqkv, B, rows, H, 0),
                        ops._t4(dqkv, B, rows, H, D), part, ops._t4(dqkv, B, rows, H, 2 * D),
                        B, H, rows, n, n_dense)
    dw = torch.zeros(128, device=DEV)
    ops.reduce_rows(part, dw)
    # fp32 reference over the valid rows
    x = qkv.float().view(B, rows, 3 * D)[:, :n].reshape(B * n, 3 * D).requires_grad_(True)
    wqf, wkf = wq.float().requires_grad_(True), wk.float().requires_grad_(True)
    fc = torch.complex(cos[:n], sin[:n])

    def nr(t, w):
        y = torch.nn.functional.rms_norm(t.view(B, n, H, 64), (64,), weight=w, eps=1e-6)
        yc = torch.view_as_complex(y.reshape(B, n, H, 32, 2)) * fc[None, :, None, :]
        return torch.view_as_real(yc).reshape(B, n, H, 64).permute(0, 2, 1, 3)
    qn, kn = nr(x[:, :D], wqf), nr(x[:, D:2 * D], wkf)
    vf = x[:, 2 * D:].view(B, n, H, 64).permute(0, 2, 1, 3)
    ref = _attn_ref(qn, kn, vf, kb[:, :n], 0.125)
    ref.backward(do.float().view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3))
    got = dqkv.float().view(B, rows, 3 * D)
    gx = x.grad.view(B, n, 3 * D)
    assert rel(got[:, :n, :D], gx[..., :D]) < 2e-2
    assert rel(got[:, :n, D:2 * D], gx[..., D:2 * D]) < 2e-2
    assert rel(got[:, :n, 2 * D:], gx[..., 2 * D:]) < 2e-2
    assert rel(dw[:64], wqf.grad) < 1e-2 and rel(dw[64:], wkf.grad) < 1e-2
    assert (got[:, n:] == sentinel).all()  # rows past n untouched
    if masked:
        dead = (kb[0, :n] == float("-inf")).nonzero().flatten()
        assert (got[0, dead, D:2 * D] == 0).all()
    # the unfused pair: same result up to the bf16 rounding of dq / dk between the two kernels
    dq2, dk2 = torch.zeros(M, D, dtype=torch.bfloat16, device=DEV), torch.zeros(M, D, dtype=torch.bfloat16, device=DEV)
    dqk = torch.zeros(M, 2 * D, dtype=torch.bfloat16, device=DEV)
    dqkv2 = torch.zeros(M, 3 * D, dtype=torch.bfloat16, device=DEV)
    ops.attn_bwd(q4, k4, v4, o4, ops._t4(do, B, rows, H), lse, delta, kb, ops._t4(dqk, B, rows, H, 0),
                 ops._t4(dqk, B, rows, H, D), ops._t4(dqkv2, B, rows, H, 2 * D), B, H, rows, n, n_dense)
    del dq2, dk2
    p2 = ops.qknorm_rope_bwd(dqk, qkv, wq, wk, cos, sin, rows, dqkv2)
    g2 = dqkv2.float().view(B, rows, 3 * D)
    assert rel(got[:, :n, :2 * D], g2[:, :n, :2 * D]) < 1e-2
    # dV: the unfused backward runs the 16x16x32 bodies, the fused one the 32x32x16 pair (its epilogue reads that
    # accumulator layout) -- the same products in another summation order
    assert rel(got[:, :n, 2 * D:], g2[:, :n, 2 * D:]) < 2e-3
    assert p2 is not None


@pytest.mark.parametrize("n,n_dense,wscale", [(1034, 1024, 1.0), (700, 520, 1.0), (4170, 4106, 1.5), (700, 520, 3.0)])
def test_attention_fwd_fixed_reference(ops, n, n_dense, wscale):
    """vpt_attn_fwd_qknorm (softmax with the QK-norm score bound as a fixed reference point instead of the running row
    maximum) vs vpt_attn_fwd (online maximum) on QK-RMSNormed, roped inputs: the same attention up to f32 / bf16
    rounding, and the -LSE both hand the backward. wscale 3 puts the bound above 60 (log2 units): the online path,
    bitwise equal to vpt_attn_fwd."""
    B, H, rows = 2, 3, ((n + 127) // 128) * 128
    D = H * 64
    qkv = rnd(B * rows, 3 * D, seed=70)
    wq = (wscale * (1 + rnd(64, scale=0.2, seed=71).float())).to(torch.bfloat16)
    wk = (wscale * (1 + rnd(64, scale=0.2, seed=72).float())).to(torch.bfloat16)
    cos, sin = _rope_tables(rows, seed=73)
    qk = ops.qknorm_rope_fwd(qkv, wq, wk, cos, sin, rows, q_scale=ops.attn_q_scale(0.125))
    kb = torch.zeros(B, rows, device=DEV)
    kb[:, n_dense + (n - n_dense) // 2:] = float("-inf")
    kb[1, n_dense:] = 0.0
    q4, k4, v4 = ops._t4(qk, B, rows, H, 0), ops._t4(qk, B, rows, H, D), ops._t4(qkv, B, rows, H, 2 * D)
    o1 = torch.zeros(B * rows, D, dtype=torch.bfloat16, device=DEV)
    o2 = torch.zeros_like(o1)
    l1 = torch.zeros(B, H, rows, device=DEV)
    l2 = torch.zeros_like(l1)
    ops.attn_fwd(q4, k4, v4, ops._t4(o1, B, rows, H), l1, kb, B, H, rows, n, n_dense)
    ops.attn_fwd_qknorm(q4, k4, v4, ops._t4(o2, B, rows, H), l2, kb, wq, wk, B, H, rows, n, n_dense)
    torch.cuda.synchronize()
    bound = 0.125 * 1.4426950408889634 * 64 * wq.float().abs().max().item() * wk.float().abs().max().item() * 1.0625
    v1 = o1.view(B, rows, D)[:, :n].float()
    v2 = o2.view(B, rows, D)[:, :n].float()
    if bound >= 60:
        assert torch.equal(v1, v2) and torch.equal(l1[..., :n], l2[..., :n])
        return
    assert rel(v2, v1) < 4e-3
    assert (l2[..., :n] - l1[..., :n]).abs().max().item() < 1e-4 * max(1.0, l1[..., :n].abs().max().item())
    # and against fp32 attention of the same (bf16) q~, k, v
    def heads(t, c0, ld):
        return t.float().view(B, rows, ld)[:, :n, c0:c0 + D].reshape(B, n, H, 64).permute(0, 2, 1, 3)
    qf = heads(qk, 0, 2 * D) / ops.attn_q_scale(0.125) * 1.0
    kf, vf = heads(qk, D, 2 * D), heads(qkv, 2 * D, 3 * D)
    ref = _attn_ref(qf, kf, vf, kb[:, :n], 0.125).permute(0, 2, 1, 3).reshape(B, n, D)
    assert rel(v2, ref) < 1e-2


@pytest.mark.parametrize("n,nk,masked", [(300, 231, False), (1000, 77, True), (64, 500, True)])
def test_cross_attention_fwd_bwd(ops, n, nk, masked):
    """SDXL cross-attention shape (src/models/sdxl/denoiser.py:101-171): n query rows attend to nk
    context rows (separate tensors); optional key mask; fp32 PyTorch reference."""
    B, H = 2, 3
    D = H * 64
    q = rnd(B * n, D, seed=60)
    kv = rnd(B * nk, 2 * D, seed=61)
    kb = torch.zeros(B, nk, device=DEV)
    n_dense = nk
    if masked:
        n_dense = nk // 2
        kb[0, nk - nk // 3:] = float("-inf")
    o = torch.zeros(B * n, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B, H, n, device=DEV)
    q_s = prescale_q(ops, q, D)  # kept alive: _t4 holds a raw pointer
    q4 = ops._t4(q_s, B, n, H, 0)
    k4 = ops._t4(kv, B, nk, H, 0)
    v4 = ops._t4(kv, B, nk, H, D)
    ops.attn_fwd(q4, k4, v4, ops._t4(o, B, n, H, 0), lse, kb, B, H, n, n, n_dense, nk=nk)

    def heads(t, rows, c0):
        return t[:, c0:c0 + D].float().view(B, rows, H, 64).permute(0, 2, 1, 3).contiguous()

    qf = heads(q, n, 0).requires_grad_(True)
    kf = heads(kv, nk, 0).requires_grad_(True)
    vf = heads(kv, nk, D).requires_grad_(True)
    ref = _attn_ref(qf, kf, vf, kb, 0.125)
    assert rel(o.view(B, n, H, 64).permute(0, 2, 1, 3), ref) < 1e-2
    do = rnd(B * n, D, seed=62)
    dq = torch.zeros(B * n, D, dtype=torch.bfloat16, device=DEV)
    dkv = torch.zeros(B * nk, 2 * D, dtype=torch.bfloat16, device=DEV)
    delta = torch.zeros(B, H, n, device=DEV)
    ops.attn_bwd(q4, k4, v4, ops._t4(o, B, n, H, 0), ops._t4(do, B, n, H, 0), lse, delta, kb, ops._t4(dq, B, n, H, 0),
                 ops._t4(dkv, B, nk, H, 0), ops._t4(dkv, B, nk, H, D), B, H, n, n, n_dense, nk=nk)
    ref.backward(do.float().view(B, n, H, 64).permute(0, 2, 1, 3))
    assert rel(dq.view(B, n, H, 64).permute(0, 2, 1, 3), qf.grad) < 2e-2
    assert rel(dkv[:, :D].reshape(B, nk, H, 64).permute(0, 2, 1, 3), kf.grad) < 2e-2
    assert rel(dkv[:, D:].reshape(B, nk, H, 64).permute(0, 2, 1, 3), vf.grad) < 2e-2


def test_attention_fwd_rescale_branch(ops):
    """Forces the online-softmax rescale branch at later tiles (guide §5.4 rule 26): query 5 meets a
    score spike at key 300 (tile 4, far past the 8-unit lazy-rescale threshold) and a smaller one at
    key 130 (tile 2, below it); full-tensor fp64 reference."""
    B, H, n = 1, 2, 400
    rows, D = 512, 2 * 64
    qkv = rnd(B * rows, 3 * D, seed=44)
    u = torch.randn(64, device=DEV)
    u = u / u.norm()
    qkv[5, 0:64] = (4.0 * u).bfloat16()
    qkv[300, D:D + 64] = (12.0 * u).bfloat16()   # score ~48 -> ~69 log2 units above the rest
    qkv[130, D:D + 64] = (1.2 * u).bfloat16()    # ~+4.8 -> 7 log2 units
    o = torch.zeros(B * rows, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.zeros(B, H, rows, device=DEV)
    qkv_s = prescale_q(ops, qkv, D)
    q4, k4, v4 = (ops._t4(qkv_s, B, rows, H, c) for c in (0, D, 2 * D))
    ops.attn_fwd(q4, k4, v4, ops._t4(o, B, rows, H, 0), lse, None, B, H, rows, n, n)

    def heads(c0):
        return qkv_s[:, c0:c0 + D].double().view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3)

    # reference on the kernel's own (pre-scaled, log2-unit) logits, so the lse bar checks arithmetic only
    s = torch.einsum("bhqd,bhkd->bhqk", heads(0), heads(D)) * math.log(2.0)
    ref = torch.einsum("bhqk,bhkd->bhqd", torch.softmax(s, -1), heads(2 * D))
    got = o.view(B, rows, H, 64)[:, :n].permute(0, 2, 1, 3).double()
    assert rel(got, ref) < 1e-2
    assert (got[0, :, 5] - ref[0, :, 5]).abs().max() < 2e-2
    ref_lse = torch.logsumexp(s, -1) / math.log(2.0)
    assert (-lse[:, :, :n].double() - ref_lse).abs().max() < 1e-3  # the kernel stores -LSE (log2)


# ------------------------------------------------------------------------------------ misc
def test_swiglu(ops):
    M, F = 300, 2048
    x12 = rnd(M, 2 * F, seed=50)
    h = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    ops.swiglu_fwd(x12, h)
    xf = x12.float().requires_grad_(True)
    ref = torch.nn.functional.silu(xf[:, :F]) * xf[:, F:]
    assert rel(h, ref) < 5e-3
    dh = rnd(M, F, seed=51)
    dx = torch.empty_like(x12)
    ops.swiglu_bwd(dh, x12, dx)
    ref.backward(dh.float())
    assert rel(dx, xf.grad) < 1e-2


@pytest.mark.parametrize("M,N", [(5000, 768), (33360, 776), (100, 4096)])
def test_bias_grad(ops, M, N):
    """Column sums (slice partials + fixed-order reduction): ragged column blocks, accumulate, and
    bitwise-repeatable back-to-back launches."""
    dy = rnd(M, N, seed=52)
    ref = dy.double().sum(0)
    out = torch.zeros(N, device=DEV)
    ops.bias_grad(dy, out)
    assert rel(out, ref) < 1e-5
    first = out.clone()
    for _ in range(3):
        ops.bias_grad(dy, out)
        assert torch.equal(out, first)  # deterministic
    ops.bias_grad(dy, out, accumulate=True)
    assert rel(out, 2 * ref) < 1e-5


@pytest.mark.parametrize("W", [96, 112, 80])  # strips of 4 + 2, 4 + 3 and 4 + 1 patches (every piece-decode width)
def test_patchify_unpatchify_roundtrip(ops, W):
    B, H = 2, 64
    img = rnd(B, 3, H, W, seed=53)
    p = torch.empty(B * (H // 16) * (W // 16), 768, dtype=torch.bfloat16, device=DEV)
    ops.patchify(img, B, H, W, p, noising=False)
    # im2col order (c, ky, kx) as Conv2d(3,128,16,16).weight.view(128,-1)
    ref = img.view(B, 3, H // 16, 16, W // 16, 16).permute(0, 2, 4, 1, 3, 5).reshape(-1, 768)
    assert torch.equal(p, ref)
    # unpatchify uses (ky, kx, c) order
    q = img.view(B, 3, H // 16, 16, W // 16, 16).permute(0, 2, 4, 3, 5, 1).reshape(-1, 768).contiguous()
    back = torch.empty_like(img)
    ops.unpatchify(q, B, H, W, back)
    assert torch.equal(back, img)


def test_noise_patchify_explicit_noise(ops):
    B, H, W = 2, 32, 48
    x = rnd(B, 3, H, W, dtype=torch.float16, seed=54)
    nz = rnd(B, 3, H, W, dtype=torch.float16, seed=55)
    t = torch.tensor([0.3, 0.8], device=DEV)
    p = torch.empty(B * (H // 16) * (W // 16), 768, dtype=torch.bfloat16, device=DEV)
    ops.patchify(x, B, H, W, p, t=t, noise=nz)
    z = (t.view(-1, 1, 1, 1) * x + (1 - t.view(-1, 1, 1, 1)) * nz).to(torch.bfloat16)
    ref = z.view(B, 3, H // 16, 16, W // 16, 16).permute(0, 2, 4, 1, 3, 5).reshape(-1, 768)
    assert rel(p, ref) < 1e-3


def test_generated_noise_is_gaussian(ops):
    B, H, W = 4, 256, 256
    x = torch.zeros(B, 3, H, W, dtype=torch.float16, device=DEV)
    t = torch.zeros(B, device=DEV)
    p = torch.empty(B * 256, 768, dtype=torch.bfloat16, device=DEV)
    ops.patchify(x, B, H, W, p, t=t, seed=1234)
    v = p.float()
    assert abs(v.mean().item()) < 0.01
    assert abs(v.std().item() - 1.0) < 0.01
    assert abs((v ** 4).mean().item() - 3.0) < 0.05


def test_generated_noise_pairs_uncorrelated(ops):
    """The two draws of a Box-Muller pair (adjacent pixels) and neighbouring pairs are uncorrelated."""
    B, H, W = 2, 256, 256
    x = torch.zeros(B, 3, H, W, dtype=torch.float16, device=DEV)
    p = torch.empty(B * 256, 768, dtype=torch.bfloat16, device=DEV)
    ops.patchify(x, B, H, W, p, t=torch.zeros(B, device=DEV), seed=99)
    v = p.float().view(-1, 2)  # (kx even, kx + 1): one pair
    assert abs(torch.corrcoef(v.t())[0, 1].item()) < 0.01
    w = p.float().view(-1, 4)  # pair j vs pair j + 1
    assert abs(torch.corrcoef(torch.stack([w[:, 0], w[:, 2]]))[0, 1].item()) < 0.01
    q = torch.empty_like(p)
    ops.patchify(x, B, H, W, q, t=torch.zeros(B, device=DEV), seed=100)
    assert abs(torch.corrcoef(torch.stack([p.float().flatten(), q.float().flatten()]))[0, 1].item()) < 0.01


def test_generated_noise_depends_on_seed_only(ops):
    """z(t) of two patchify calls with one seed use the same noise: z(0.5) = bf16(0.5 x + 0.5 eps) with eps from
    z(0) (bf16-rounded there, hence the tolerance); the velocity loss with in-kernel noise is reproducible."""
    B, H, W = 2, 64, 96
    np_ = (H // 16) * (W // 16)
    x = rnd(B, 3, H, W, dtype=torch.float16, seed=70)
    z0 = torch.empty(B * np_, 768, dtype=torch.bfloat16, device=DEV)
    z5 = torch.empty_like(z0)
    ops.patchify(x, B, H, W, z0, t=torch.zeros(B, device=DEV), seed=4242)
    ops.patchify(x, B, H, W, z5, t=torch.full((B,), 0.5, device=DEV), seed=4242)
    xp = x.view(B, 3, H // 16, 16, W // 16, 16).permute(0, 2, 4, 1, 3, 5).reshape(-1, 768).float()
    assert (z5.float() - (0.5 * xp + 0.5 * z0.float())).abs().max().item() < 0.03
    t = torch.tensor([0.3, 0.75], device=DEV)
    pred = rnd(B * np_, 768, seed=71)
    outs = []
    for _ in range(2):
        d = torch.empty_like(pred)
        part = torch.empty(ops.loss_blocks(), device=DEV)
        loss = torch.empty(1, device=DEV)
        ops.flow_loss(pred, x, t, B, H, W, d, part, loss, target=1, seed=4242)
        outs.append((loss.clone(), d))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("target", [0, 1, 2])
@pytest.mark.parametrize("B,H,W", [(2, 64, 32), (2, 48, 112), (9, 512, 1024)])  # ragged strips; > 4096 strips
def test_flow_loss(ops, target, B, H, W):
    np_ = (H // 16) * (W // 16)
    x = rnd(B, 3, H, W, dtype=torch.float16, seed=56)
    nz = rnd(B, 3, H, W, dtype=torch.float16, seed=57)
    t = torch.linspace(0.2, 0.99, B, device=DEV)
    pred_img = rnd(B, 3, H, W, seed=58)
    pred = torch.empty(B * np_, 768, dtype=torch.bfloat16, device=DEV)
    ops.unpatchify(pred, B, H, W, pred_img, reverse=True)
    dpred = torch.empty_like(pred)
    part = torch.empty(ops.loss_blocks(), device=DEV)
    loss = torch.empty(1, device=DEV)
    ops.flow_loss(pred, x, t, B, H, W, dpred, part, loss, target=target, noise=nz)
    pf = pred_img.float().requires_grad_(True)
    if target == 0:
        ref = torch.nn.functional.mse_loss(pf, x.float())
    elif target == 2:  # velocity prediction: target = clean - noise as the reference's fp16 tensors (class_to_image:151)
        ref = torch.nn.functional.mse_loss(pf, (x - nz).float())
    else:
        tt = t.view(-1, 1, 1, 1)
        z = tt * x.float() + (1 - tt) * nz.float()
        c = (1 - tt).clamp_min(0.05)
        ref = torch.nn.functional.mse_loss((pf - z) / c, (x.float() - z) / c)
    ref.backward()
    assert abs(loss.item() - ref.item()) / ref.item() < 1e-5
    dimg = torch.empty_like(pred_img)
    ops.unpatchify(dpred, B, H, W, dimg)
    assert rel(dimg, pf.grad) < 5e-3


def test_timestep_embed(ops):
    vals = torch.tensor([0.0, 0.5, 0.123, 1.0, 256.0, 1024.0, 7.0], device=DEV)
    out = torch.empty(vals.numel(), 256, dtype=torch.bfloat16, device=DEV)
    ops.timestep_embed(vals, out)
    half = 128
    fr = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=DEV) / half)
    a = vals[:, None] * fr[None]
    ref = torch.cat([torch.cos(a), torch.sin(a)], -1)
    assert (out.float() - ref).abs().max().item() < 1e-2


def test_assemble_disassemble(ops):
    B, np_, n_ctx = 2, 16, 8
    rows = np_ + 10 + n_ctx
    patches, size_emb = rnd(B * np_, 768, seed=60), rnd(B * 6, 768, seed=61)
    time_emb, tpe, ctx = rnd(B, 768, seed=62), rnd(4, 768, seed=63), rnd(B * n_ctx, 768, seed=64)
    x = torch.empty(B * rows, 768, dtype=torch.bfloat16, device=DEV)
    ops.assemble_tokens(patches, size_emb, time_emb, tpe, ctx, n_ctx, B, np_, rows, x)
    xv = x.view(B, rows, 768)
    assert torch.equal(xv[:, :np_].reshape(-1, 768), patches)
    assert torch.equal(xv[:, np_:np_ + 6].reshape(-1, 768), size_emb)
    tt = (time_emb.view(B, 1, 768) + tpe.view(1, 4, 768)).to(torch.bfloat16)
    assert torch.equal(xv[:, np_ + 6:np_ + 10], tt)
    assert torch.equal(xv[:, np_ + 10:].reshape(-1, 768), ctx)
    dx = rnd(B * rows, 768, seed=65)
    dp, ds = torch.empty_like(patches), torch.empty_like(size_emb)
    dt, dtpe = torch.empty_like(time_emb), torch.empty(4, 768, device=DEV)
    ops.disassemble_tokens(dx, B, np_, rows, dp, ds, dt, dtpe)
    dxv = dx.view(B, rows, 768)
    assert torch.equal(dp, dxv[:, :np_].reshape(-1, 768))
    assert rel(dt, dxv[:, np_ + 6:np_ + 10].float().sum(1)) < 5e-3
    assert rel(dtpe, dxv[:, np_ + 6:np_ + 10].float().sum(0)) < 1e-5
    # ctx-rows backward: dctx += the context rows of dx (f32 accumulation over context blocks), and
    # those rows of dx are cleared; run twice to check the accumulation
    ctx_ref = dxv[:, np_ + 10:].float().reshape(-1, 768).clone()
    prior = torch.randn(B * n_ctx, 768, device=DEV)
    dctx = prior.clone()
    ops.ctx_rows(dx, B, np_ + 10, rows, n_ctx, dctx=dctx, backward=True)
    torch.testing.assert_close(dctx, prior + ctx_ref, rtol=0, atol=1e-6)
    assert dx.view(B, rows, 768)[:, np_ + 10:].abs().sum().item() == 0
    assert torch.equal(dx.view(B, rows, 768)[:, :np_ + 10], dxv[:, :np_ + 10])


def test_embedding(ops):
    V, D = 50, 768
    table = rnd(V + 1, D, seed=70)
    ids = torch.tensor([[1, 5, 5, 50], [0, 2, 50, 50]], device=DEV)
    out = torch.empty(8, D, dtype=torch.bfloat16, device=DEV)
    ops.embed_gather(table, ids, out)
    assert torch.equal(out, table[ids.view(-1)])
    dr = rnd(8, D, seed=71)
    dt = torch.zeros(V + 1, D, device=DEV)
    ops.embed_scatter_add(dr, ids, V, dt)
    ref = torch.zeros(V + 1, D, device=DEV).index_add_(0, ids.view(-1), dr.float())
    ref[V] = 0
    assert rel(dt, ref) < 1e-6


@pytest.mark.parametrize("case", ["mixed", "one_row_hot", "empty", "out_of_range", "large"])
@pytest.mark.parametrize("accumulate", [False, True])
def test_embed_grad_set(ops, case, accumulate):
    """vpt_embed_grad_set against index_add (float64): duplicates, the padding id (no gradient), ids past the table
    (ignored), R = 0, every id in one 8-row block (the per-block position lists are O(R), not a rank sort) and the
    largest R; overwrite (the whole table written, zeros elsewhere) and accumulate (old + sum on the named rows, the
    others untouched); bitwise reproducible."""
    V, D = 45, 768  # table rows V + 1 (the padding row V), 6 blocks of 8 rows (the last one ragged)
    g = torch.Generator().manual_seed(5)
    R = {"mixed": 64, "one_row_hot": 4096, "empty": 0, "out_of_range": 32, "large": 16384}[case]
    if case == "one_row_hot":
        ids = torch.full((R,), 3)
        ids[::7] = 4
    else:
        ids = torch.randint(0, V + 1, (R,), generator=g)
    if case == "out_of_range":
        ids[::5] = V + 3
    ids = ids.to(DEV)
    dr = rnd(max(R, 1), D, seed=72)[:R]
    old = rnd(V + 1, D, dtype=torch.float32, seed=73)
    outs = []
    for _ in range(2):
        dt = old.clone()
        ops.embed_grad_set(dr, ids, V, dt, accumulate=accumulate)
        outs.append(dt)
    assert torch.equal(outs[0], outs[1])
    keep = (ids >= 0) & (ids < V)
    s = torch.zeros(V + 1, D, dtype=torch.float64, device=DEV).index_add_(0, ids[keep], dr[keep].double())
    named = torch.zeros(V + 1, dtype=torch.bool, device=DEV)
    named[ids[keep]] = True
    ref = torch.where(named[:, None], old.double() + s, old.double()) if accumulate else s
    err = (outs[0].double() - ref).abs().max().item()
    assert err <= 1e-6 * max(1.0, ref.abs().max().item()) * max(1, R) ** 0.5, err
    assert torch.equal(outs[0][V], old[V] if accumulate else torch.zeros_like(old[V]))


def test_gauss_noise_is_the_in_kernel_draw(ops):
    """vpt_gauss_noise writes exactly the noise patchify generates (patchify at t = 0 outputs bf16(eps))."""
    B, H, W = 2, 64, 96
    x = rnd(B, 3, H, W, dtype=torch.float16, seed=80)
    nz = ops.gauss_noise(torch.empty(B, 3, H, W, dtype=torch.float16, device=DEV), 777)
    a = torch.empty(B * (H // 16) * (W // 16), 768, dtype=torch.bfloat16, device=DEV)
    b = torch.empty_like(a)
    t = torch.tensor([0.0, 0.6], device=DEV)
    ops.patchify(x, B, H, W, a, t=t, seed=777)
    ops.patchify(x, B, H, W, b, t=t, noise=nz)
    assert torch.equal(a, b)


@pytest.mark.parametrize("k,H,W", [(2, 64, 96), (4, 128, 64), (2, 1088, 960)])
@pytest.mark.parametrize("explicit", [False, True])
def test_area_lowres(ops, k, H, W, explicit):
    """vpt_area_lowres vs F.interpolate(mode="area", scale_factor=1/k) of the fp16 image, the fp16 noise and the f32
    noisy image (arb_class_to_image.py:233-245): image / noise within one fp16 rounding, z within one bf16 rounding."""
    import torch.nn.functional as F
    B = 2
    x = rnd(B, 3, H, W, dtype=torch.float16, seed=81)
    t = torch.tensor([0.25, 0.9], device=DEV)
    nz = rnd(B, 3, H, W, dtype=torch.float16, seed=82) if explicit else \
        ops.gauss_noise(torch.empty(B, 3, H, W, dtype=torch.float16, device=DEV), 4321)
    h, w = H // k, W // k
    il = torch.empty(B, 3, h, w, dtype=torch.float16, device=DEV)
    nl, zl = torch.empty_like(il), torch.empty(B, 3, h, w, dtype=torch.bfloat16, device=DEV)
    ops.area_lowres(x, B, H, W, k, t, il, nl, zl, noise=nz if explicit else None, seed=4321)

    def area(v):
        return F.interpolate(v.float(), scale_factor=1.0 / k, mode="area")
    tt = t.view(-1, 1, 1, 1)
    assert (il.float() - area(x)).abs().max().item() <= 1e-3
    assert (nl.float() - area(nz)).abs().max().item() <= 2e-3
    zr = area(tt * x.float() + (1 - tt) * nz.float())
    assert ((zl.float() - zr).abs() <= zr.abs() * 2 ** -8 + 1e-6).all()


# ------------------------------------------------------------------------------------ RAdamScheduleFree
@pytest.mark.parametrize("gb", [False, True])
@pytest.mark.parametrize("adam", [0, 1])
def test_radam_sf_step_vector_path_bitwise_equals_scalar(ops, gb, adam):
    """radam_sf_step runs 4 elements per thread when y / z / v / grad are aligned for it and one per thread
    otherwise: the same update on the same values, once aligned and once at a 1-element offset (scalar path),
    must agree bit for bit -- weight decay, both clippings, grad_scale and a ragged tail included."""
    n = 100_003
    g0 = torch.Generator().manual_seed(11)
    y = (torch.randn(n, generator=g0) * 0.1).to(torch.bfloat16)
    z = torch.randn(n, generator=g0) * 0.1
    v = torch.rand(n, generator=g0) * 1e-3
    g = torch.randn(n, generator=g0)
    gdt = torch.bfloat16 if gb else torch.float32
    coef = torch.tensor([0.7], device=DEV)
    outs = []
    for off in (0, 1):
        def place(t, dt):
            buf = torch.zeros(n + 1, dtype=dt, device=DEV)
            buf[off:off + n] = t.to(dt).to(DEV)
            return buf[off:off + n]
        yy, zz, vv, gg = place(y, torch.bfloat16), place(z, torch.float32), place(v, torch.float32), place(g, gdt)
        ops.radam_sf_step(yy, gg, zz, vv, beta2=0.999, bias_correction2=0.3, eps=1e-8, ckp1=0.2, adaptive_y_lr=-1e-3,
                          lr=2e-3, decay=0.01, grad_scale=0.5, adam=adam, clip_coef=coef, clip_value=0.3)
        outs.append((yy.cpu(), zz.cpu(), vv.cpu()))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32),
                           b.view(torch.int16) if b.dtype == torch.bfloat16 else b.view(torch.int32))


@pytest.mark.parametrize("decay,silent", [(0.0, True), (0.05, False)])
def test_radam_schedulefree_steps_vs_restatement(ops, decay, silent):
    """The fused optimizer (vpt.optim over radam_sf_step / sf_lerp / sf_init kernels) against the CPU
    restatement of schedulefree 1.4.1 (tests/sf_reference.py; the package is absent, parity unpinned):
    25 steps through the silent-SGD warm-up (rho_t <= 4 for steps 1-5) into rectified Adam, with
    weight decay, a grad_scale fold (DDP mean), ranges applied piecewise, and the train()/eval()
    swap the reference trainer drives (src/trainer/common.py:276-285) in the middle."""
    from tests.sf_reference import SFRef
    from vpt.optim import RAdamScheduleFreeFlat
    n = 70_001  # odd: a partial last block
    g0 = torch.Generator().manual_seed(5)
    y0 = (torch.randn(n, generator=g0) * 0.1).to(torch.bfloat16)
    y_gpu = y0.to(DEV)
    gr_gpu = torch.zeros(n, device=DEV)
    opt = RAdamScheduleFreeFlat(y_gpu, gr_gpu, lr=3e-3, weight_decay=decay, silent_sgd_phase=silent)
    y_ref = y0.clone()
    ref = SFRef([y_ref], lr=3e-3, weight_decay=decay, silent_sgd_phase=silent)
    opt.train()
    ref.train()
    scale = 0.5
    for k in range(25):
        g = torch.randn(n, generator=g0) * (1.0 + 0.1 * k)
        gr_gpu.copy_(g.to(DEV) / scale)  # the kernel folds grad_scale (e.g. 1/world) in
        s = opt.begin_step()
        opt.apply_range(s, 0, 30_000, grad_scale=scale)
        opt.apply_range(s, 30_000, n, grad_scale=scale)
        opt.end_step(s)
        rs = ref.step([g])
        assert math.isclose(opt.param_groups[0]["scheduled_lr"], rs["lr"], rel_tol=1e-12, abs_tol=1e-30)
        if k == 12:  # an eval()/train() round trip, as around a checkpoint or preview
            opt.eval()
            ref.eval()
            assert (y_gpu.cpu().float() - y_ref.float()).abs().max().item() <= 2 ** -7 * y_ref.float().abs().max().item()
            opt.train()
            ref.train()
    torch.cuda.synchronize()
    # f32 state: the same algorithm in a different op order; bf16 y may round differently by 1 ulp
    torch.testing.assert_close(opt.z.cpu(), ref.z[0], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(opt.v.cpu(), ref.v[0], rtol=1e-4, atol=1e-10)
    yd = (y_gpu.cpu().float() - y_ref.float()).abs()
    ulp = y_ref.float().abs().clamp_min(1e-3) * 2 ** -7
    assert (yd <= ulp).float().mean().item() > 0.999, (yd / ulp).max().item()
    assert opt.param_groups[0]["k"] == 25 and ref.group["k"] == 25
    if silent:  # steps 1-5 moved nothing but v
        assert opt.param_groups[0]["lr_max"] > 0
