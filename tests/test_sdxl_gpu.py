"""GPU parity of the SDXL QLoRA kernels and block, all compute in
libvpt_hip.so: LayerNorm / GeGLU against PyTorch (fp32 math; bf16 graph for GeGLU), NF4 dequant
bit-exact against the oracle restatement, NF4 quantize against the oracle, and the full LoRA-trained
TransformerBlock (forward + backward) against the reference's own native-bf16 run
(tests/golden/sdxl_block.safetensors). Tolerances are stated per test."""

import json
import os

import pytest
import torch
from safetensors import safe_open
from safetensors.torch import load_file

from oracle import sdxl_oracle as SO

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(__file__), "golden", "sdxl_block.safetensors")


@pytest.fixture(scope="module")
def ops():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vpt import ops as o
    return o


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * scale).bfloat16()


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def cos(a, b):
    a, b = a.double().cpu().reshape(-1), b.double().cpu().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,D", [(333, 640), (70, 1280), (5, 2048)])
def test_layernorm_fwd_bwd(ops, M, D):
    x = rnd(M, D, seed=1)
    w = (1 + rnd(D, scale=0.1, seed=2).float()).bfloat16()
    b = rnd(D, scale=0.1, seed=3)
    y, mean, rstd = ops.layernorm_fwd(x, w, b)
    xf, wf, bf = (t.float().requires_grad_(True) for t in (x, w, b))
    ref = torch.nn.functional.layer_norm(xf, (D,), wf, bf, eps=1e-5)
    assert rel(y, ref) < 5e-3
    dy = rnd(M, D, seed=4)
    dres = rnd(M, D, seed=5)
    nb = ops.layernorm_bwd_blocks(M)
    dwp = torch.empty(nb, D, device=DEV)
    dbp = torch.empty(nb, D, device=DEV)
    dx = ops.layernorm_bwd(dy, x, mean, rstd, w, dres=dres, dw_part=dwp, db_part=dbp)
    ref.backward(dy.float())
    assert rel(dx.float() - dres.float(), xf.grad) < 1e-2
    assert rel(dwp.sum(0), wf.grad) < 1e-4 and rel(dbp.sum(0), bf.grad) < 1e-4


def test_geglu_matches_bf16_graph(ops):
    """out = h * gelu(gate) and its autograd on the bf16 graph (denoiser.py:174-186)."""
    M, F = 300, 640
    x12 = rnd(M, 2 * F, seed=6)
    out = ops.geglu_fwd(x12)
    xr = x12.clone().requires_grad_(True)
    h, g = xr.chunk(2, dim=-1)
    ref = h * torch.nn.functional.gelu(g)
    assert rel(out, ref) < 1e-3 and (out != ref.detach()).float().mean().item() < 1e-3
    dy = rnd(M, F, seed=7)
    ref.backward(dy)
    dx = ops.geglu_bwd(dy, x12)
    assert rel(dx, xr.grad) < 2e-3


def test_nf4_dequant_bit_exact(ops):
    g = torch.Generator().manual_seed(8)
    w = torch.randn(1280, 640, generator=g) * 0.05
    st = SO.nf4_quantize(w)
    ref = SO.nf4_dequantize(st).to(torch.bfloat16)
    d = {k: v.to(DEV) for k, v in st.items()}
    out = torch.empty(1280, 640, dtype=torch.bfloat16, device=DEV)
    ops.nf4_dequant(d["packed"], d["qabsmax"], d["absmax2"].float(), d["code2"], d["offset"], w.numel(), out)
    assert torch.equal(out.cpu(), ref)


def test_nf4_quantize_matches_oracle(ops):
    """Codes and nested statistics of quantize_4bit (restated) from the same bf16 weights. The offset
    (mean of absmax) is summed in a different order (~1e-8 relative), and the signed dynamic map is
    exponentially dense near 0, so nested codes of near-offset absmax values may land on a neighbouring
    code: compare the DECODED absmax (what dequantisation uses), not the raw nested codes."""
    from vpt.sdxl import NF4Weight
    g = torch.Generator().manual_seed(9)
    w = (torch.randn(640, 2560, generator=g) * 0.03).bfloat16()
    ref = SO.nf4_quantize(w.float())
    q = NF4Weight.quantize(w.to(DEV), SO.dynamic_map())
    assert torch.equal(q.packed.cpu(), ref["packed"])
    mine = {"qabsmax": q.qabsmax.cpu(), "absmax2": q.absmax2.cpu(), "offset": q.offset.cpu(), "code2": ref["code2"]}
    am_ref = SO.nf4_absmax(ref)
    assert ((SO.nf4_absmax(mine) - am_ref).abs() <= 1e-5 * am_ref.abs().max()).all()
    assert abs(q.offset.item() - ref["offset"].item()) < 1e-6 * abs(ref["offset"].item()) + 1e-9
    assert torch.allclose(q.absmax2.cpu(), ref["absmax2"], rtol=1e-5)
    # dequantize() emits bf16 (what the GEMM consumes): compare with the oracle rounded the same way;
    # the only remaining differences come from the ~1e-5 absmax deviations above flipping a rounding
    deq = q.dequantize().float().cpu()
    assert rel(deq, SO.nf4_dequantize(ref).bfloat16().float()) < 1e-3


@pytest.mark.parametrize("forward", [True, False])
@pytest.mark.parametrize("lora", [False, True])
def test_gemm_nf4_bit_exact_vs_dequant_gemm(ops, forward, lora):
    """vpt_gemm_nf4 (dequant inside the GEMM, LoRA as an extra K tile) == vpt_nf4_dequant + the T128 bf16
    GEMM over the concatenated operands [A | lora_a] . [W | lora_b] (same MFMA order: bit-exact), at a
    partial M tile, 5 N tiles and both weight orientations."""
    from vpt.sdxl import NF4Weight
    Nw, Kw, M, r = 1280, 640, 300, 16
    g = torch.Generator().manual_seed(12)
    st = SO.nf4_quantize(torch.randn(Nw, Kw, generator=g) * 0.05)
    w = NF4Weight.from_state(dict(st, shape=torch.tensor([Nw, Kw])))
    Wd = w.dequantize()
    N, K = (Nw, Kw) if forward else (Kw, Nw)
    a = rnd(M, K, seed=13)
    la = rnd(M, r, scale=0.5, seed=14) if lora else None
    lb = (rnd(N, r, scale=0.1, seed=15) if forward else rnd(r, N, scale=0.1, seed=15)) if lora else None
    bias = rnd(N, scale=0.1, seed=16) if forward else None
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm_nf4(a, w, forward, out, lora_a=la, lora_b=lb, bias=bias)
    # reference: one dense GEMM over K + 64 (the LoRA tile zero-padded to 64 k), T128 geometry
    pad = 64
    a2 = torch.zeros(M, K + pad, dtype=torch.bfloat16, device=DEV)
    a2[:, :K] = a
    if forward:
        b2 = torch.zeros(N, K + pad, dtype=torch.bfloat16, device=DEV)
        b2[:, :K] = Wd
        if lora:
            a2[:, K:K + r] = la
            b2[:, K:K + r] = lb
        ref = torch.empty_like(out)
        ops.gemm(a2 if lora else a, True, b2 if lora else Wd, True, M, N, K + (pad if lora else 0), ref, bias=bias,
                 geometry=128)
    else:
        b2 = torch.zeros(K + pad, N, dtype=torch.bfloat16, device=DEV)
        b2[:K] = Wd
        if lora:
            a2[:, K:K + r] = la
            b2[K:K + r] = lb
        ref = torch.empty_like(out)
        ops.gemm(a2 if lora else a, True, b2 if lora else Wd, False, M, N, K + (pad if lora else 0), ref, geometry=128)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()


@pytest.mark.parametrize("geometry,splits", [(128, 1), (256, 1), (256, 3), (128, 2)])
@pytest.mark.parametrize("forward", [True, False])
@pytest.mark.parametrize("r", [16, 48])
def test_gemm_lora_bit_exact_vs_concatenated_gemm(ops, geometry, splits, forward, r):
    """vpt_gemm_bf16_lora (the LoRA term as a K-extension of the base GEMM) == one bf16 GEMM of the same
    geometry over the concatenated operands [A | A2 | 0] . [B | B2 | 0] (the extension tile zero-padded to the
    geometry's K step: 64 for T128, 32 for the ring): the same MFMA sequence, so bit-exact. Partial M and N
    tiles, bias and residual epilogues; r = 48 is three adapters side by side (a block-diagonal B2). Split-K (the
    extension in the last slice, bias / residual in the slab reduce) equals the same split of the concatenated GEMM."""
    M, Nw, Kw = 600, 1280, 640
    N, K = (Nw, Kw) if forward else (Kw, Nw)
    W = rnd(Nw, Kw, scale=0.05, seed=30)
    a = rnd(M, K, seed=31)
    a2 = rnd(M, r, scale=0.5, seed=32)
    b2 = rnd(N, r, scale=0.1, seed=33) if forward else rnd(r, N, scale=0.1, seed=33)
    bias = rnd(N, scale=0.1, seed=34) if forward else None
    resid = rnd(M, N, seed=35)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm_lora(a, W, forward, a2, b2, M, N, K, out, bias=bias, resid=resid, geometry=geometry, splits=splits)
    step = 64 if geometry == 128 else 32
    pad = (r + step - 1) // step * step
    ac = torch.zeros(M, K + pad, dtype=torch.bfloat16, device=DEV)
    ac[:, :K], ac[:, K:K + r] = a, a2
    if forward:
        bc = torch.zeros(N, K + pad, dtype=torch.bfloat16, device=DEV)
        bc[:, :K], bc[:, K:K + r] = W, b2
    else:
        bc = torch.zeros(K + pad, N, dtype=torch.bfloat16, device=DEV)
        bc[:K], bc[K:K + r] = W, b2
    ref = torch.empty_like(out)
    if splits == 1:
        ops.gemm(ac, True, bc, forward, M, N, K + pad, ref, bias=bias, resid=resid, geometry=geometry)
    else:  # the same K slices: the concatenated K split at the base GEMM's slice length
        sl = ((K + splits - 1) // splits + 63) // 64 * 64
        parts = [(k0, min(K, k0 + sl)) for k0 in range(0, K, sl)]
        acc = torch.zeros(M, N, dtype=torch.float32, device=DEV)
        for i, (k0, k1) in enumerate(parts):
            last = i == len(parts) - 1
            kk = slice(k0, (K + pad) if last else k1)
            sl_out = torch.empty(M, N, dtype=torch.float32, device=DEV)
            ops.gemm(ac[:, kk].contiguous(), True, (bc[:, kk] if forward else bc[kk]).contiguous(), forward, M, N,
                     (K + pad if last else k1) - k0, sl_out, out_mode=ops.OUT_F32, geometry=geometry)
            acc += sl_out
        y = acc + (bias.float() if bias is not None else 0.0)
        ref = (y.bfloat16().float() + resid.float()).bfloat16()
    torch.cuda.synchronize()
    if splits == 1:
        assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()
    else:  # slab sum order (z = 0, 1, ...) equals the += order above; per-slice MFMA order as the slice GEMM
        assert rel(out, ref) < 1e-3
    # and against fp32 math: bf16(bf16(A.B + bias + A2.B2) + resid)
    Bf = W.float() if forward else W.float().t()
    B2f = b2.float() if forward else b2.float().t()
    y = a.float() @ Bf.t() + a2.float() @ B2f.t() + (bias.float() if bias is not None else 0.0)
    assert rel(out.float() - resid.float(), y) < 1e-2


@pytest.mark.parametrize("forward", [True, False])
@pytest.mark.parametrize("M,Nw,Kw", [(4224, 1280, 1280), (600, 1280, 640), (1000, 640, 1280)])
def test_gemm_lora_r2_128_equals_t128(ops, forward, M, Nw, Kw):
    """The config-5 LoRA GEMMs on geometry 1281 (128x128 tiles, R2 pipeline, the K-extension padded to 32) == geometry
    128 (the extension padded to 64 with zeros): equal outputs, bias and residual epilogues, forward and input gradient;
    the grouped form (q | k | v) as well."""
    N, K = (Nw, Kw) if forward else (Kw, Nw)
    W = rnd(Nw, Kw, scale=0.05, seed=60)
    a = rnd(M, K, seed=61)
    a2 = rnd(M, 16, scale=0.5, seed=62)
    b2 = rnd(N, 16, scale=0.1, seed=63) if forward else rnd(16, N, scale=0.1, seed=63)
    bias = rnd(N, scale=0.1, seed=64) if forward else None
    resid = rnd(M, N, seed=65)
    ref = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    ops.gemm_lora(a, W, forward, a2, b2, M, N, K, ref, bias=bias, resid=resid, geometry=128, splits=1)
    ops.gemm_lora(a, W, forward, a2, b2, M, N, K, out, bias=bias, resid=resid, geometry=1281, splits=1)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()
    if forward:
        Ws = [rnd(Nw, Kw, scale=0.03, seed=66 + g) for g in range(3)]
        ups = [rnd(Nw, 16, scale=0.1, seed=70 + g) for g in range(3)]
        ds = rnd(M, 48, scale=0.5, seed=73)
        o1 = torch.empty(M, 3 * Nw, dtype=torch.bfloat16, device=DEV)
        o2 = torch.full((M, 3 * Nw), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.gemm_lora_grouped(a, torch.cat(Ws, 0), ds, ups, o1, geometry=128, splits=1)
        ops.gemm_lora_grouped(a, torch.cat(Ws, 0), ds, ups, o2, geometry=1281, splits=1)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2)


@pytest.mark.parametrize("gn,geometry", [(1280, 128), (1280, 256), (640, 128)])
def test_gemm_lora_grouped_bit_exact_vs_per_target(ops, gn, geometry):
    """vpt_gemm_bf16_lora_grouped (q | k | v of one input as one GEMM, each column block with its own LoRA term)
    == three vpt_gemm_bf16_lora calls of the same geometry, column block by column block (bit-exact)."""
    M, K, r = 700, 1280, 16
    x = rnd(M, K, seed=50)
    Ws = [rnd(gn, K, scale=0.03, seed=51 + g) for g in range(3)]
    ups = [rnd(gn, r, scale=0.1, seed=55 + g) for g in range(3)]
    ds = rnd(M, 3 * r, scale=0.5, seed=59)
    out = torch.empty(M, 3 * gn, dtype=torch.bfloat16, device=DEV)
    ops.gemm_lora_grouped(x, torch.cat(Ws, 0), ds, ups, out, geometry=geometry)
    for g in range(3):
        ref = torch.empty(M, gn, dtype=torch.bfloat16, device=DEV)
        ops.gemm_lora(x, Ws[g], True, ds[:, g * r:(g + 1) * r].contiguous(), ups[g], M, gn, K, ref, geometry=geometry,
                      splits=1)
        torch.cuda.synchronize()
        assert torch.equal(out[:, g * gn:(g + 1) * gn], ref), g


def test_sdxl_block_fused_qkv_matches_per_target(ops, monkeypatch):
    """The block's fused q|k|v GEMMs (forward and input gradient) against the per-target LoRALinear path on the same
    weights and inputs: output, input / context gradients and every adapter gradient within bf16 rounding (the
    fused input gradient sums the three projections' contributions in f32 before one rounding)."""
    from vpt import sdxl
    fx, d, sd = _block_inputs()
    res = []
    for fuse in (True, False):
        blk = sdxl.SDXLTransformerBlock(d["dim"], d["heads"], d["context_dim"], d["rank"], d["alpha"], sd)
        for t in sdxl.TARGETS:  # non-zero ups so every adapter term is live
            blk.lin[t].up = rnd(*blk.lin[t].up.shape, scale=0.05, seed=70 + sdxl.TARGETS.index(t))
        if not fuse:
            monkeypatch.setattr(blk, "_fuse_qkv", lambda Wb: False)
        B, n, nc = 2, 80, 20
        x = rnd(B * n, d["dim"], seed=60)
        ctx = rnd(B * nc, d["context_dim"], seed=61)
        y = blk.forward(x, ctx, B, n, nc)
        dx, dctx = blk.backward(rnd(B * n, d["dim"], scale=0.1, seed=62))
        torch.cuda.synchronize()
        res.append((y, dx, dctx, {t: (blk.lin[t].g_up.clone(), blk.lin[t].g_down.clone()) for t in sdxl.TARGETS}))
    (y0, dx0, c0, g0), (y1, dx1, c1, g1) = res
    assert torch.equal(y0, y1)  # the grouped forward is per-column-block identical
    assert rel(dx0, dx1) < 5e-3 and rel(c0, c1) < 5e-3
    for t in sdxl.TARGETS:
        assert rel(g0[t][0], g1[t][0]) < 5e-3 and rel(g0[t][1], g1[t][1]) < 5e-3, t


@pytest.mark.parametrize("mode", ["dequant", "resident", "inline"])
def test_lora_linear_nf4_base_modes_agree(ops, mode):
    """The three ways the NF4 base enters the GEMM (vpt.sdxl.BASE_MODES) on one LoRA target at the config-5
    1280-channel shape: "dequant" (bitsandbytes MatMul4Bit: dequantise per call, bf16 GEMM) and "resident" are
    bitwise identical; "inline" (dequant inside the GEMM) agrees to bf16 rounding of differently ordered sums."""
    from vpt.sdxl import LoRALinearNF4, NF4Weight
    g = torch.Generator().manual_seed(40)
    st = SO.nf4_quantize(torch.randn(1280, 1280, generator=g) * 0.03)
    base = NF4Weight.from_state(dict(st, shape=torch.tensor([1280, 1280])))
    down, up = rnd(16, 1280, scale=0.05, seed=41), rnd(1280, 16, scale=0.05, seed=42)
    bias = rnd(1280, scale=0.1, seed=43)
    x, dy, res = rnd(4096, 1280, seed=44), rnd(4096, 1280, seed=45), rnd(4096, 1280, seed=46)
    out = []
    for md in ("dequant", mode):
        lin = LoRALinearNF4(base, bias, down, up, alpha=1.0, rank=16, base_mode=md)
        y = lin.forward(x, resid=res)
        dx = lin.backward(dy)
        out.append((y, dx, lin.g_up.clone(), lin.g_down.clone()))
    for u, v in zip(*out):
        if mode == "inline":
            assert rel(u, v) < 5e-3
        else:
            assert torch.equal(u, v)
    # the dequant path against fp32 math on the oracle's dequantised base
    W = SO.nf4_dequantize(st).bfloat16().float().to(DEV)
    ds = (x.float() @ down.float().t() * (1.0 / 16)).bfloat16().float()
    yr = x.float() @ W.t() + bias.float() + ds @ up.float().t()
    assert rel(out[0][0].float() - res.float(), yr) < 1e-2


def test_lora_linear_nf4_fused_vs_dequant_path(ops):
    """The fused LoRALinearNF4 path and the dequant-to-scratch path agree (same math, one vs three bf16
    roundings of the LoRA sum): rel <= 1e-2 on y, dx and both adapter grads, at SDXL's 640 / 2048 widths."""
    from vpt.sdxl import LoRALinearNF4, NF4Weight
    g = torch.Generator().manual_seed(17)
    st = SO.nf4_quantize(torch.randn(640, 2048, generator=g) * 0.03)
    base = NF4Weight.from_state(dict(st, shape=torch.tensor([640, 2048])))
    down, up = rnd(16, 2048, scale=0.05, seed=18), rnd(640, 16, scale=0.05, seed=19)
    bias = rnd(640, scale=0.1, seed=20)
    x, dy = rnd(700, 2048, seed=21), rnd(700, 640, seed=22)
    res = []
    for fused in (True, False):
        lin = LoRALinearNF4(base, bias, down, up, alpha=16.0, rank=16)
        lin.fused = fused
        y = lin.forward(x)
        dx = lin.backward(dy)
        res.append((y, dx, lin.g_up.clone(), lin.g_down.clone()))
    for u, v in zip(*res):
        assert rel(u, v) < 1e-2


def _block_inputs():
    with safe_open(GOLD, "pt") as f:
        d = json.loads(f.metadata()["dims"])
    fx = load_file(GOLD)
    sd = SO.make_block_weights(d["dim"], d["heads"], d["context_dim"], d["rank"], seed=d["weight_seed"])
    for t in SO.LORA_TARGETS:
        sd[f"{t}.linear.weight"] = {k.split("/")[-1]: v for k, v in fx.items() if k.startswith(f"nf4/{t}/")}
    return fx, d, sd


def test_lora_linear_nf4_matches_oracle(ops):
    """a29: y = linear(x) + s * up(down(x)) over the NF4-dequantised base, and its adapter/input grads,
    vs the fp32 oracle (lora.py:92-104); bf16 bar rel <= 2e-2, grads cos >= 0.999."""
    from vpt.sdxl import LoRALinearNF4, NF4Weight
    fx, d, sd = _block_inputs()
    t = "ff.net.0.proj"
    lin = LoRALinearNF4(NF4Weight.from_state(sd[f"{t}.linear.weight"]), sd[f"{t}.linear.bias"].to(DEV).bfloat16(),
                        sd[f"{t}.lora_down.weight"].to(DEV), sd[f"{t}.lora_up.weight"].to(DEV), d["alpha"], d["rank"])
    x = rnd(300, d["dim"], seed=10)
    y = lin.forward(x)
    dy = rnd(300, y.shape[1], seed=11)
    dx = lin.backward(dy)
    W = SO.nf4_dequantize(sd[f"{t}.linear.weight"])
    wr = {f"{t}.linear.weight": W, f"{t}.linear.bias": sd[f"{t}.linear.bias"].bfloat16().float(),
          f"{t}.lora_down.weight": sd[f"{t}.lora_down.weight"].bfloat16().float().requires_grad_(True),
          f"{t}.lora_up.weight": sd[f"{t}.lora_up.weight"].bfloat16().float().requires_grad_(True)}
    xr = x.float().cpu().requires_grad_(True)
    yr = SO.lora_linear(xr, wr, t, d["rank"], d["alpha"])
    yr.backward(dy.float().cpu())
    assert rel(y, yr) < 2e-2
    assert rel(dx, xr.grad) < 2e-2
    assert cos(lin.g_down, wr[f"{t}.lora_down.weight"].grad) > 0.999
    assert cos(lin.g_up, wr[f"{t}.lora_up.weight"].grad) > 0.999


def test_sdxl_block_matches_reference_bf16():
    """a30: the LoRA-trained TransformerBlock, forward + backward, vs the reference's own native-bf16
    run (TransformerBlock + LoRALinear, NF4-dequantised bases). Bars: output rel-L2 <= 2e-2, input /
    context grads <= 3e-2, every adapter grad norm within 5 % and cosine >= 0.99."""
    from vpt.sdxl import SDXLTransformerBlock
    fx, d, sd = _block_inputs()
    blk = SDXLTransformerBlock(d["dim"], d["heads"], d["context_dim"], d["rank"], d["alpha"], sd)
    B, n, nc = d["B"], d["n"], d["nc"]
    x = fx["x"].to(DEV).bfloat16().reshape(B * n, -1).contiguous()
    c = fx["ctx"].to(DEV).bfloat16().reshape(B * nc, -1).contiguous()
    y = blk.forward(x, c, B, n, nc)
    dx, dctx = blk.backward(fx["dy"].to(DEV).bfloat16().reshape(B * n, -1).contiguous())
    torch.cuda.synchronize()
    assert rel(y, fx["bf16/out"].reshape(B * n, -1)) < 2e-2
    assert rel(dx, fx["bf16/dx"].reshape(B * n, -1)) < 3e-2
    assert rel(dctx, fx["bf16/dctx"].reshape(B * nc, -1)) < 3e-2
    grads = blk.lora_grads()
    bad = []
    for k, v in fx.items():
        if not k.startswith("bf16/grad/"):
            continue
        name = k[len("bf16/grad/"):]
        g = grads[name].cpu()
        if abs(g.norm() - v.norm()) > 0.05 * v.norm() or cos(g, v) < 0.99:
            bad.append((name, g.norm().item(), v.norm().item(), cos(g, v)))
    assert not bad, bad


def test_sdxl_spatial_transformer_matches_reference_bf16():
    """SpatialTransformer (denoiser.py:283-365): GroupNorm, NF4 proj_in / proj_out, 2 LoRA blocks, residual,
    forward + backward vs the reference's own native-bf16 run (tests/golden/sdxl_spatial.safetensors).
    Bars: output rel-L2 <= 2e-2, input / context grads <= 3e-2, adapter grads norm within 5 %, cos >= 0.99."""
    from vpt.sdxl import SDXLSpatialTransformer
    path = os.path.join(os.path.dirname(__file__), "golden", "sdxl_spatial.safetensors")
    with safe_open(path, "pt") as f:
        d = json.loads(f.metadata()["dims"])
    fx = load_file(path)
    C, heads, depth, cdim, rank, alpha = d["C"], d["heads"], d["depth"], d["context_dim"], d["rank"], d["alpha"]
    B, H, W, nc = d["B"], d["H"], d["W"], d["nc"]
    sd = SO.make_spatial_weights(C, heads, depth, cdim, rank, seed=d["weight_seed"])
    for k in list(sd):
        if k.endswith(".linear.weight") or k in ("proj_in.weight", "proj_out.weight"):
            sd[k] = {kk.split("/")[-1]: v for kk, v in fx.items() if kk.startswith(f"nf4/{k}/")}
    st = SDXLSpatialTransformer(C, heads, depth, cdim, rank, alpha, sd)
    HW = H * W
    x = fx["x"].to(DEV).bfloat16().reshape(B, C, HW).contiguous()
    c = fx["ctx"].to(DEV).bfloat16().reshape(B * nc, cdim).contiguous()
    y = st.forward(x, c, B, HW, nc)
    dx, dctx = st.backward(fx["dy"].to(DEV).bfloat16().reshape(B, C, HW).contiguous())
    torch.cuda.synchronize()
    assert rel(y, fx["bf16/out"].reshape(B, C, HW)) < 2e-2
    assert rel(y, fx["fp32/out"].reshape(B, C, HW)) < 2e-2
    assert rel(dx, fx["bf16/dx"].reshape(B, C, HW)) < 3e-2
    assert rel(dctx, fx["bf16/dctx"].reshape(B * nc, cdim)) < 3e-2
    grads = st.lora_grads()
    bad = []
    for k, v in fx.items():
        if not k.startswith("bf16/grad/"):
            continue
        name = k[len("bf16/grad/"):]
        g = grads[name].cpu()
        if abs(g.norm() - v.norm()) > 0.05 * v.norm() or cos(g, v) < 0.99:
            bad.append((name, g.norm().item(), v.norm().item(), cos(g, v)))
    assert not bad and len(grads) == 2 * 10 * depth, bad


@pytest.mark.parametrize("B,C,HW", [(2, 640, 4096), (3, 1280, 1024), (2, 640, 56 * 72), (2, 1280, 28 * 36),
                                    (1, 1280, 24 * 44)])
def test_groupnorm_and_transpose(ops, B, C, HW):
    """GroupNorm(32, C, eps 1e-6) fwd / input-grad (frozen affine) vs torch fp32, and the NCHW<->token
    transposes (bit-exact) with the residual add, at SDXL's two stage shapes of the square 1024^2 bucket and of the
    896x1152 / 768x1408 buckets (HW not a multiple of the 64 x 64 transpose tile)."""
    G = 32
    x = rnd(B, C, HW, seed=30)
    w = (1 + rnd(C, scale=0.1, seed=31).float()).bfloat16()
    b = rnd(C, scale=0.1, seed=32)
    y, mean, rstd = ops.groupnorm_fwd(x, w, b, B, C, G, HW)
    xf = x.float().requires_grad_(True)
    ref = torch.nn.functional.group_norm(xf, G, w.float(), b.float(), eps=1e-6)
    assert rel(y, ref) < 5e-3
    dy, dres = rnd(B, C, HW, seed=33), rnd(B, C, HW, seed=34)
    dx = ops.groupnorm_bwd(dy, x, mean, rstd, w, B, C, G, HW, dres=dres)
    ref.backward(dy.float())
    assert rel(dx.float() - dres.float(), xf.grad) < 1e-2
    t = ops.transpose_add(x, B, C, HW)
    assert torch.equal(t, x.transpose(1, 2).contiguous())
    back = ops.transpose_add(t, B, HW, C, add=dres)
    assert torch.equal(back, (x.float() + dres.float()).bfloat16())


def test_sdxl_stacks_step_binds_flat_adapters(ops):
    """C5 step plumbing (vpt.sdxl_train): two reduced stacks (640 / 1280 channels, one block, 16x16 and 8x8
    latents); the flat gradient buffer is exactly the stacks' adapter gradients, up-projection grads are
    non-zero and down-projection grads are exactly zero at LoRA's zero-initialised up (lora.py:71-84), the
    context gradient is finite, and the fused optimizer runs."""
    from vpt.sdxl_train import SDXLStacksQLoRA
    m = SDXLStacksQLoRA(B=2, stacks=[("a", 640, 10, 1, 16), ("b", 1280, 20, 1, 8)], n_ctx=77, seed=3)
    xs, ctx, gs = m.make_inputs(seed=4)
    dctx = m.step(xs, ctx, gs)
    torch.cuda.synchronize()
    assert torch.isfinite(dctx.float()).all() and dctx.float().abs().sum() > 0
    seen = 0
    for (_, _, _, st) in m.stacks:
        for k, g in st.lora_grads().items():
            assert g.data_ptr() >= m.grads.data_ptr() and g.numel() > 0
            seen += g.numel()
            if "lora_down" in k:
                assert g.abs().max().item() == 0.0, k
            else:
                assert g.abs().max().item() > 0, k
    assert seen == m.grads.numel() == m.n_adapter_params()
    assert m.flops_per_step() > 0


def test_sdxl_stacks_precomputed_ctx_kv_matches_per_block(ops, monkeypatch):
    """SDXLStacksQLoRA.precompute_ctx_kv (every block's cross-attention k / v of the fixed context as stacked GEMMs,
    two width classes) against the per-block projections: the same step with non-zero adapters gives the same
    context gradient and adapter gradients to bf16 rounding of differently ordered sums (the stacked GEMM's
    k / v are bit-identical in exact arithmetic; ds = s * ctx . down^T is one GEMM instead of lora_proj)."""
    from vpt.sdxl_train import SDXLStacksQLoRA
    res = []
    for pre in (True, False):
        m = SDXLStacksQLoRA(B=2, stacks=[("a", 640, 10, 1, 16), ("b", 1280, 20, 2, 8), ("c", 640, 10, 1, 16)],
                            n_ctx=77, seed=3)
        g = torch.Generator(device=DEV).manual_seed(9)
        with torch.no_grad():
            m.params.copy_((torch.randn(m.params.shape, device=DEV, generator=g) * 0.03).bfloat16())
        if not pre:
            monkeypatch.setattr(m, "precompute_ctx_kv", lambda ctx, save=True: False)
        xs, ctx, gs = m.make_inputs(seed=4)
        m.opt.step = lambda: None  # compare gradients, not the update
        dctx = m.step(xs, ctx, gs)
        torch.cuda.synchronize()
        res.append((dctx.float().clone(), m.grads.clone()))
    (c0, g0), (c1, g1) = res
    assert rel(c0, c1) < 1e-2
    assert rel(g0, g1) < 1e-2 and cos(g0, g1) > 0.9999


@pytest.mark.parametrize("M,K,N", [(16384, 640, 5120), (1000, 1280, 2048), (924, 2048, 1280)])
def test_lora_skinny_kernels_vs_torch(ops, M, K, N):
    """vpt_lora_proj (both W layouts) and vpt_lora_wgrad (both output layouts, accumulate) vs fp32 torch on
    the same bf16 operands: rel <= 5e-3 (bf16 output rounding) / 1e-5 (f32 sums)."""
    x, dy = rnd(M, K, seed=40), rnd(M, N, seed=41)
    down, up = rnd(16, K, scale=0.05, seed=42), rnd(N, 16, scale=0.05, seed=43)
    ds = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj(x, down, True, ds, alpha=0.5)
    assert rel(ds, 0.5 * x.float() @ down.float().t()) < 5e-3
    vs = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj(dy, up, False, vs, alpha=2.0)
    assert rel(vs, 2.0 * dy.float() @ up.float()) < 5e-3
    g_up = torch.full((N, 16), 0.25, device=DEV)
    g_down = torch.full((16, K), -0.5, device=DEV)
    ops.lora_wgrad2(dy, ds, g_up, x, vs, g_down, accumulate=True, alpha=3.0)
    assert rel(g_up, 0.25 + 3.0 * dy.float().t() @ ds.float()) < 1e-5
    assert rel(g_down, -0.5 + 3.0 * vs.float().t() @ x.float()) < 1e-5
    ops.lora_wgrad2(dy, ds, g_up, x, vs, g_down, accumulate=False)
    assert rel(g_up, dy.float().t() @ ds.float()) < 1e-5 and rel(g_down, vs.float().t() @ x.float()) < 1e-5
    # batched reduces (lora_wgrad_batch: split-M slabs per target, one reduce launch per 32 jobs): bit-identical
    # to the per-target path, over 52 targets with distinct inputs (4 flushes: workspace names are re-issued
    # after each, so a slab still pending reduction must never be handed out again) and a flush forced by a
    # change of alpha
    T = 52
    dss = [ds.roll(i, 0) for i in range(T)]
    vss = [vs.roll(-i, 0) for i in range(T)]
    gu = [torch.full((N, 16), 0.25, device=DEV) for _ in range(T)]
    gd = [torch.full((16, K), -0.5, device=DEV) for _ in range(T)]
    with ops.lora_wgrad_batch():
        for i in range(T - 1):
            ops.lora_wgrad2(dy, dss[i], gu[i], x, vss[i], gd[i], accumulate=True, alpha=3.0)
        ops.lora_wgrad2(dy, dss[T - 1], gu[T - 1], x, vss[T - 1], gd[T - 1], accumulate=False)
    for i in range(T):
        ref_u, ref_d = torch.full((N, 16), 0.25, device=DEV), torch.full((16, K), -0.5, device=DEV)
        last = i == T - 1
        ops.lora_wgrad2(dy, dss[i], ref_u, x, vss[i], ref_d, accumulate=not last, alpha=1.0 if last else 3.0)
        assert torch.equal(gu[i], ref_u) and torch.equal(gd[i], ref_d), i


@pytest.mark.parametrize("w_kmajor", [True, False])
def test_lora_proj_grouped_bit_exact_vs_per_group(ops, w_kmajor):
    """vpt_lora_proj_grouped (the q / k / v adapters of one input, or of the three column blocks of the q|k|v
    gradient) against one vpt_lora_proj per group on the same operands: bit-identical."""
    M, D = 1000, 1280
    if w_kmajor:  # forward: one input, the three downs stacked [3 * 16][D]
        x = rnd(M, D, seed=90)
        w = rnd(3 * 16, D, scale=0.05, seed=91)
        xs = [x, x, x]
        ws = [w[16 * g:16 * (g + 1)] for g in range(3)]
        x_goff, w_goff = 0, 16 * D
    else:  # input gradient: [dq | dk | dv] [M][3D], the three ups stacked [3 * D][16]
        x = rnd(M, 3 * D, seed=92)
        w = rnd(3 * D, 16, scale=0.05, seed=93)
        xs = [x[:, g * D:(g + 1) * D] for g in range(3)]
        ws = [w[g * D:(g + 1) * D] for g in range(3)]
        x_goff, w_goff = D, D * 16
    out = torch.empty(M, 48, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj_grouped(x if w_kmajor else x[:, :D], x_goff, ws[0], w_goff, 3, w_kmajor, out, alpha=0.0625)
    for g in range(3):
        ref = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
        ops.lora_proj(xs[g], ws[g], w_kmajor, ref, alpha=0.0625)
        assert torch.equal(out[:, 16 * g:16 * (g + 1)], ref), g


def test_lora_wgrad_deferred_batch_matches_immediate(ops, monkeypatch):
    """lora_wgrad_batch with the slab products deferred to one vpt_lora_wgrad_partial_batch launch (jobs of
    different M and widths, as a transformer block's self-attention, cross-attention context and ff targets) is
    bit-identical to each target's own slab launch."""
    shapes = [(4096, 1280, 1280), (924, 1280, 2048), (4096, 10240, 1280), (4096, 1280, 5120), (1000, 640, 640)]
    ops_in = []
    for i, (M, n_out, n_in) in enumerate(shapes):
        ops_in.append((rnd(M, n_out, seed=100 + i), rnd(M, 16, seed=110 + i), rnd(M, n_in, seed=120 + i),
                       rnd(M, 16, seed=130 + i)))
    res = []
    for defer in (True, False):
        monkeypatch.setattr(ops, "_LORA_DEFER", defer)
        gs = [(torch.full((n_out, 16), 0.5, device=DEV), torch.full((16, n_in), -0.25, device=DEV))
              for (_, n_out, n_in) in shapes]
        with ops.lora_wgrad_batch():
            for (dy, ds, x, vs), (gu, gd) in zip(ops_in, gs):
                ops.lora_wgrad2(dy, ds, gu, x, vs, gd, accumulate=True, alpha=0.0625)
        torch.cuda.synchronize()
        res.append(gs)
    for i, ((a_u, a_d), (b_u, b_d)) in enumerate(zip(*res)):
        assert torch.equal(a_u, b_u) and torch.equal(a_d, b_d), shapes[i]
    dy, ds, x, vs = ops_in[1]
    assert rel(res[0][1][0], 0.5 + 0.0625 * dy.float().t() @ ds.float()) < 1e-5


@pytest.mark.parametrize("M,D,G", [(4100, 1280, 3), (1000, 640, 1), (77, 1280, 1)])
def test_layernorm_lora_fwd_bit_exact(ops, M, D, G):
    """vpt_layernorm_lora_fwd: y / mean / rstd bit-identical to vpt_layernorm_fwd and ds to vpt_lora_proj(_grouped) on
    that y (the separate launches it replaces), M not a multiple of the kernel's 16 rows."""
    x = rnd(M, D, seed=140)
    w, b = rnd(D, scale=0.5, seed=141) + 1.0, rnd(D, scale=0.1, seed=142)
    w = w.to(torch.bfloat16)
    down = rnd(16 * G, D, scale=0.05, seed=143)
    ds = torch.empty(M, 16 * G, dtype=torch.bfloat16, device=DEV)
    y, m, r = ops.layernorm_lora_fwd(x, w, b, down, G, 0.0625, ds)
    y0, m0, r0 = ops.layernorm_fwd(x, w, b)
    assert torch.equal(y, y0) and torch.equal(m, m0) and torch.equal(r, r0)
    ref = torch.empty(M, 16 * G, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj_grouped(y0, 0, down[:16], 16 * D, G, True, ref, alpha=0.0625)
    assert torch.equal(ds, ref)


def test_sdxl_block_fused_ln_lora_bitwise(ops, monkeypatch):
    """The blocks with their LayerNorms fused to the LoRA down-projections (norm1 -> q|k|v, norm2 -> attn2.to_q,
    norm3 -> ff.net.0.proj) give a step bit-identical to the unfused one: context gradient and every adapter
    gradient (flat adapter layout of SDXLStacksQLoRA, where the q|k|v downs are adjacent), both widths."""
    from vpt import sdxl
    from vpt.sdxl_train import SDXLStacksQLoRA
    res = []
    for fused in (True, False):
        monkeypatch.setattr(sdxl, "FUSED_LN_LORA", fused)
        m = SDXLStacksQLoRA(B=2, stacks=[("a", 640, 10, 1, 16), ("b", 1280, 20, 1, 8)], n_ctx=77, seed=3)
        g = torch.Generator(device=DEV).manual_seed(9)
        with torch.no_grad():
            m.params.copy_((torch.randn(m.params.shape, device=DEV, generator=g) * 0.03).bfloat16())
        xs, ctx, gs = m.make_inputs(seed=4)
        m.opt.step = lambda: None  # compare gradients, not the update
        dctx = m.step(xs, ctx, gs)
        torch.cuda.synchronize()
        res.append((dctx.clone(), m.grads.clone()))
    (c0, g0), (c1, g1) = res
    assert torch.equal(c0, c1) and torch.equal(g0, g1)


def test_sdxl_stack_fused_ln_bwd_prev_bitwise(ops, monkeypatch):
    """Two-block stacks: each block's norm1 backward emitting the previous block's ff.net.2 input-gradient LoRA operand
    (FUSED_LN_BWD_PREV, ops.layernorm_bwd_lora) gives a step bit-identical to the separate lora_proj."""
    from vpt import sdxl
    from vpt.sdxl_train import SDXLStacksQLoRA
    res = []
    for fused in (True, False):
        monkeypatch.setattr(sdxl, "FUSED_LN_BWD_PREV", fused)
        m = SDXLStacksQLoRA(B=2, stacks=[("a", 640, 10, 2, 16), ("b", 1280, 20, 2, 8)], n_ctx=77, seed=3)
        g = torch.Generator(device=DEV).manual_seed(9)
        with torch.no_grad():
            m.params.copy_((torch.randn(m.params.shape, device=DEV, generator=g) * 0.03).bfloat16())
        xs, ctx, gs = m.make_inputs(seed=4)
        m.opt.step = lambda: None  # compare gradients, not the update
        dctx = m.step(xs, ctx, gs)
        torch.cuda.synchronize()
        res.append((dctx.clone(), m.grads.clone()))
    (c0, g0), (c1, g1) = res
    assert torch.equal(c0, c1) and torch.equal(g0, g1)


def test_nf4_dequant_batch_bit_exact(ops):
    """vpt_nf4_dequant_batch (several tensors of different sizes in one launch, the last block of each partial)
    against the oracle's dequantisation of each: bit-identical."""
    from vpt.sdxl import NF4Weight
    g = torch.Generator().manual_seed(11)
    shapes = [(1280, 640), (640, 2048), (1280, 1280), (320, 64), (2560, 640)]
    pairs, refs = [], []
    for (o, i) in shapes:
        st = SO.nf4_quantize(torch.randn(o, i, generator=g) * 0.05)
        refs.append(SO.nf4_dequantize(st).to(torch.bfloat16))
        w = NF4Weight.from_state(dict(st, shape=torch.tensor([o, i])))
        pairs.append((w, torch.full((o, i), float("nan"), dtype=torch.bfloat16, device=DEV)))
    outs = ops.nf4_dequant_batch(pairs)
    for out, ref in zip(outs, refs):
        assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("M,D", [(4100, 1280), (333, 640)])
def test_layernorm_bwd_no_partials_bit_exact(ops, M, D):
    """The frozen-affine LayerNorm backward (no dw / db partials: one row per wave, dres in flight with x and dy)
    gives dx bit-identical to the partial-producing form."""
    x, dy, dres = rnd(M, D, seed=170), rnd(M, D, seed=171), rnd(M, D, seed=172)
    w = (rnd(D, scale=0.5, seed=173) + 1.0).to(torch.bfloat16)
    b = rnd(D, scale=0.1, seed=174)
    _, mean, rstd = ops.layernorm_fwd(x, w, b)
    nb = ops.layernorm_bwd_blocks(M)
    dwp = torch.empty(nb, D, device=DEV)
    dbp = torch.empty(nb, D, device=DEV)
    dx0 = ops.layernorm_bwd(dy, x, mean, rstd, w, dres=dres, dw_part=dwp, db_part=dbp)
    dx1 = ops.layernorm_bwd(dy, x, mean, rstd, w, dres=dres)
    dx2 = ops.layernorm_bwd(dy, x, mean, rstd, w)
    dx3 = ops.layernorm_bwd(dy, x, mean, rstd, w, dw_part=dwp, db_part=dbp)
    assert torch.equal(dx0, dx1) and torch.equal(dx2, dx3)


@pytest.mark.parametrize("M,D,res", [(4100, 1280, True), (333, 640, False)])
def test_layernorm_bwd_lora_bit_exact(ops, M, D, res):
    """vpt_layernorm_bwd_lora: dx bit-identical to vpt_layernorm_bwd and vs to vpt_lora_proj(dx, up, w_kmajor=0)."""
    x, dy = rnd(M, D, seed=180), rnd(M, D, seed=181)
    dres = rnd(M, D, seed=182) if res else None
    w = (rnd(D, scale=0.5, seed=183) + 1.0).to(torch.bfloat16)
    b = rnd(D, scale=0.1, seed=184)
    up = rnd(D, 16, scale=0.05, seed=185)
    _, mean, rstd = ops.layernorm_fwd(x, w, b)
    vs = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    dx = ops.layernorm_bwd_lora(dy, x, mean, rstd, w, up, 0.0625, vs, dres=dres)
    dx0 = ops.layernorm_bwd(dy, x, mean, rstd, w, dres=dres)
    assert torch.equal(dx, dx0)
    ref = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj(dx0, up, False, ref, alpha=0.0625)
    assert torch.equal(vs, ref)


@pytest.mark.parametrize("gn,geometry", [(1280, 128), (1280, 256), (640, 128)])
def test_gemm_lora_scaled_columns(ops, gn, geometry):
    """vpt_gemm_bf16_lora(_grouped)_scaled: alpha = 2^-3 on columns [0, gn) is exact scaling, so the output equals
    the unscaled GEMM's with the first column block times 2^-3 and the rest untouched (bit-exact); a general alpha
    (the attention q scale) matches fp32 math within one bf16 rounding."""
    M, K, r = 700, 1280, 16
    x = rnd(M, K, seed=150)
    Ws = [rnd(gn, K, scale=0.03, seed=151 + g) for g in range(3)]
    ups = [rnd(gn, r, scale=0.1, seed=155 + g) for g in range(3)]
    ds = rnd(M, 3 * r, scale=0.5, seed=159)
    W = torch.cat(Ws, 0)
    base = torch.empty(M, 3 * gn, dtype=torch.bfloat16, device=DEV)
    ops.gemm_lora_grouped(x, W, ds, ups, base, geometry=geometry)
    out = torch.empty_like(base)
    ops.gemm_lora_grouped(x, W, ds, ups, out, geometry=geometry, alpha=0.125, alpha_cols=gn)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :gn], (base[:, :gn].float() * 0.125).bfloat16())
    assert torch.equal(out[:, gn:], base[:, gn:])
    # single target, every column scaled
    one = torch.empty(M, gn, dtype=torch.bfloat16, device=DEV)
    ops.gemm_lora(x, Ws[0], True, ds[:, :r].contiguous(), ups[0], M, gn, K, one, geometry=geometry, alpha=0.125)
    torch.cuda.synchronize()
    assert torch.equal(one, out[:, :gn])
    # general alpha vs fp32
    a = ops.attn_q_scale(0.125)
    ops.gemm_lora(x, Ws[0], True, ds[:, :r].contiguous(), ups[0], M, gn, K, one, geometry=geometry, alpha=a)
    y = (x.float() @ Ws[0].float().t() + ds[:, :r].float() @ ups[0].float().t()) * a
    torch.cuda.synchronize()
    assert rel(one, y) < 1e-2
    assert (one.float() - y).abs().max().item() <= y.abs().max().item() * 2 ** -7


@pytest.mark.parametrize("M,F", [(4224, 5120), (333, 2560), (77, 640), (16, 128)])
def test_geglu_fwd_lora(ops, M, F):
    """vpt_geglu_fwd_lora: out bit-identical to vpt_geglu_fwd; ds = alpha * out . down^T within bf16 rounding of
    vpt_lora_proj (another f32 summation order) and of fp32 math; repeated launches (the tickets reset) bit-identical."""
    x12 = rnd(M, 2 * F, seed=193)
    down = rnd(16, F, scale=0.05, seed=194)
    ds = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    out = ops.geglu_fwd_lora(x12, down, 0.0625, ds)
    ref = ops.geglu_fwd(x12)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    dref = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj(ref, down, True, dref, alpha=0.0625)
    y = (ref.float() @ down.float().t()) * 0.0625
    torch.cuda.synchronize()
    assert rel(ds, y) < 5e-3 and rel(ds, dref) < 5e-3
    assert (ds.float() - dref.float()).abs().max().item() <= y.abs().max().item() * 2 ** -6
    for _ in range(3):
        ds2 = torch.full((M, 16), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.geglu_fwd_lora(x12, down, 0.0625, ds2)
        torch.cuda.synchronize()
        assert torch.equal(ds2, ds)


@pytest.mark.parametrize("M,F", [(4100, 5120), (4224, 5120), (333, 2560), (77, 640), (16, 128)])
def test_geglu_bwd_lora(ops, M, F):
    """vpt_geglu_bwd_lora: dx12 bit-identical to vpt_geglu_bwd; vs = alpha * dx12 . up within bf16 rounding of
    vpt_lora_proj (another f32 summation order) and of fp32 math. F = 640: 5 chunk pairs over 2 blocks of 4 waves
    (idle waves); repeated launches on one workspace (the tickets reset) give bit-identical vs."""
    dy, x12 = rnd(M, F, seed=190), rnd(M, 2 * F, seed=191)
    up = rnd(2 * F, 16, scale=0.05, seed=192)
    vs = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    dx12 = ops.geglu_bwd_lora(dy, x12, up, 0.0625, vs)
    ref = ops.geglu_bwd(dy, x12)
    torch.cuda.synchronize()
    assert torch.equal(dx12, ref)
    for _ in range(3):
        vs2 = torch.full((M, 16), float("nan"), dtype=torch.bfloat16, device=DEV)
        ops.geglu_bwd_lora(dy, x12, up, 0.0625, vs2)
        torch.cuda.synchronize()
        assert torch.equal(vs2, vs)
    vref = torch.empty(M, 16, dtype=torch.bfloat16, device=DEV)
    ops.lora_proj(ref, up, False, vref, alpha=0.0625)
    y = (ref.float() @ up.float()) * 0.0625
    torch.cuda.synchronize()
    assert rel(vs, y) < 5e-3 and rel(vs, vref) < 5e-3
    assert (vs.float() - vref.float()).abs().max().item() <= y.abs().max().item() * 2 ** -6
