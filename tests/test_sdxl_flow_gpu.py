"""GPU parity of BASELINE config 5 as a flow-matching step (vpt.sdxl_flow, all compute in libvpt_hip.so):

- the step's own kernels against PyTorch on the same bf16 tensors: noising (prepare_scaled_noised_latents,
  src/modules/loss/flow_match.py:60-74), velocity MSE and its gradient (flow_match.py:85-96), the sinusoidal
  embeddings of t * 1000 and the size conditions, pixel (un)shuffle -- bit-exact or f32-rounding bars;
- the whole step (timestep -> noise -> conditioning -> 11 stacks with skips -> velocity loss -> backward) on a
  reduced SDXL topology against the fp32 oracle (oracle/sdxl_oracle.flow_match_loss, built on the
  SpatialTransformer restatement that tests/golden/sdxl_spatial.safetensors pins to the reference);
- the stacks at production shapes against the same oracle: one 640-channel SpatialTransformer (2 blocks, 64 x 64
  latents, 231 x 2048 context) and one 1280-channel block at 32 x 32, with the NF4 bases the step uses
  (NF4 values themselves are parity-unpinned: bitsandbytes is absent).
Bars (bf16 compute vs fp32): outputs rel-L2 <= 2e-2 (3e-2 after 11 stacks), loss rel <= 1e-2, adapter gradients
norm within 5 % and cosine >= 0.99 (0.98 after 11 stacks)."""

import math
import os

import pytest
import torch
import torch.nn.functional as F

from oracle import sdxl_oracle as SO

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.set_num_threads(min(16, os.cpu_count() or 1))


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, device=DEV, generator=g) * scale).bfloat16()


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def cos(a, b):
    a, b = a.double().cpu().reshape(-1), b.double().cpu().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


# ----------------------------------------------------------------------------------------- kernels
def test_flow_noise_matches_reference_arithmetic():
    """eps given: z = t x + (1 - t) eps in f32 (t is an f32 tensor) then bf16 -- bit-exact vs torch; generated
    noise: standard normal (moments), stored bf16, and z consistent with it; clean_at_zero swaps the weights."""
    from vpt import ops
    B = 3
    x = rnd(B, 4, 32, 48, seed=1)
    eps = rnd(B, 4, 32, 48, seed=2)
    t = torch.tensor([0.1, 0.5, 0.93], device=DEV)
    z = torch.empty_like(x)
    ops.flow_noise(x, t, B, z, eps_in=eps)
    tt = t.view(B, 1, 1, 1)
    assert torch.equal(z, (tt * x + (1 - tt) * eps).bfloat16())
    ops.flow_noise(x, t, B, z, eps_in=eps, clean_at_zero=True)
    assert torch.equal(z, ((1 - tt) * x + tt * eps).bfloat16())
    big = rnd(4, 4, 128, 128, seed=3)
    t4 = torch.full((4,), 0.25, device=DEV)
    zb, eb = torch.empty_like(big), torch.empty_like(big)
    ops.flow_noise(big, t4, 4, zb, eps=eb, seed=7)
    e = eb.float()
    assert abs(e.mean().item()) < 5e-3 and abs(e.std().item() - 1) < 5e-3
    assert torch.equal(zb, (0.25 * big.float() + 0.75 * e).bfloat16())
    zb2, eb2 = torch.empty_like(big), torch.empty_like(big)
    ops.flow_noise(big, t4, 4, zb2, eps=eb2, seed=8)
    assert not torch.equal(eb, eb2)  # another step, another draw
    ops.flow_noise(big, t4, 4, zb2, eps=eb2, noise_scale=2.0, seed=7)
    assert torch.equal(eb2, (eb.float() * 2).bfloat16())


def test_velocity_loss_and_grad_match_torch():
    """mse(v, eps - x) under autocast: target rounded to bf16 (bf16 tensor subtraction), f32 mean; gradient
    2 (v - target) / n in bf16."""
    from vpt import ops
    v, x, eps = rnd(4, 4, 64, 64, seed=4), rnd(4, 4, 64, 64, seed=5), rnd(4, 4, 64, 64, seed=6)
    loss = torch.zeros(1, device=DEV)
    dv = torch.empty_like(v)
    ops.velocity_loss(v, x, eps, loss, dv)
    vf = v.float().requires_grad_(True)
    ref = F.mse_loss(vf, (eps - x).float())
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * ref.item()
    assert rel(dv, vf.grad) < 4e-3  # bf16 rounding of the gradient


@pytest.mark.parametrize("dim", [320, 256])
def test_sinusoid_embed_matches_oracle(dim):
    from vpt import ops
    t = torch.tensor([0.0, 1.0, 37.5, 999.0, 512.0, 1024.0], device=DEV)
    out = ops.sinusoid_embed(t, dim)
    assert (out.float().cpu() - SO.sinusoid(t.cpu(), dim)).abs().max().item() < 8e-3  # bf16 output


@pytest.mark.parametrize("C,H,W,r", [(4, 128, 128, 2), (640, 64, 64, 2), (3, 8, 12, 4)])
def test_space_to_depth_is_pixel_unshuffle(C, H, W, r):
    from vpt import ops
    x = rnd(2, C, H, W, seed=9)
    tok = ops.space_to_depth(x, 2, C, H, W, r)
    ref = F.pixel_unshuffle(x, r).permute(0, 2, 3, 1).reshape(2, (H // r) * (W // r), C * r * r)
    assert torch.equal(tok, ref)
    back = ops.space_to_depth(tok, 2, C, H, W, r, inverse=True)
    assert torch.equal(back, x)


# ----------------------------------------------------------------------------------------- the step
def _export_stack(st):
    """Oracle weights (fp32, CPU) of a HIP SDXLSpatialTransformer: NF4 bases dequantised by the oracle's own
    restatement from the device states, LoRA adapters as the bf16 values the step trains."""
    def nf4(w):
        return SO.nf4_dequantize({"packed": w.packed.cpu(), "qabsmax": w.qabsmax.cpu(), "absmax2": w.absmax2.cpu(),
                                  "code2": w.code2.cpu(), "offset": w.offset.cpu(), "shape": torch.tensor(w.shape)})
    w = {"norm.weight": st.norm_w.float().cpu(), "norm.bias": st.norm_b.float().cpu(),
         "proj_in.weight": nf4(st.proj_in.base), "proj_in.bias": st.proj_in.bias.float().cpu(),
         "proj_out.weight": nf4(st.proj_out.base), "proj_out.bias": st.proj_out.bias.float().cpu()}
    for i, blk in enumerate(st.blocks):
        pre = f"transformer_blocks.{i}."
        for t, lin in blk.lin.items():
            w[pre + f"{t}.linear.weight"] = nf4(lin.base)
            if lin.bias is not None:
                w[pre + f"{t}.linear.bias"] = lin.bias.float().cpu()
            for k, p in (("lora_down", lin.down), ("lora_up", lin.up)):
                w[pre + f"{t}.{k}.weight"] = p.float().cpu().requires_grad_(True)
        for n in ("norm1", "norm2", "norm3"):
            w[pre + f"{n}.weight"] = blk.norm[n][0].float().cpu()
            w[pre + f"{n}.bias"] = blk.norm[n][1].float().cpu()
    return w


def _grad_pairs(st):
    """(oracle name, HIP f32 gradient) of every adapter of a stack."""
    return [(f"transformer_blocks.{i}.{t}.{k}.weight", (l.g_down if k == "lora_down" else l.g_up).cpu())
            for i, blk in enumerate(st.blocks) for t, l in blk.lin.items() for k in ("lora_down", "lora_up")]


def _check_adapter_grads(pairs, w, min_cos, norm_tol=5e-2):
    bad = []
    for name, g in pairs:
        ref = w[name].grad
        if ref is None or ref.norm() < 1e-12:
            continue
        c = cos(g, ref)
        if abs(g.norm().item() - ref.norm().item()) > norm_tol * ref.norm().item() or c < min_cos:
            bad.append((name, round(g.norm().item(), 6), round(ref.norm().item(), 6), round(c, 5)))
    return bad


@pytest.mark.parametrize("latent", [(32, 32), (32, 48), (48, 32)])
def test_flow_match_step_matches_oracle_reduced_topology(latent):
    """The whole config-5 step on SDXL's topology at reduced sizes (latent 32 x 32: level A 128 ch at 16 x 16, level B
    256 ch at 8 x 8; and the non-square buckets 32 x 48 / 48 x 32; one block per stack, context 20 x 128) with random
    (non-zero) LoRA adapters: velocity loss, prediction and every adapter gradient vs the fp32 oracle on the same t,
    noise and weights."""
    from vpt.sdxl_flow import SDXLFlowMatchQLoRA
    stacks = [("down.A.0", 128, 2, 1, 16), ("down.A.1", 128, 2, 1, 16), ("down.B.0", 256, 4, 1, 8),
              ("down.B.1", 256, 4, 1, 8), ("mid.B", 256, 4, 1, 8), ("up.B.0", 256, 4, 1, 8), ("up.B.1", 256, 4, 1, 8),
              ("up.B.2", 256, 4, 1, 8), ("up.A.0", 128, 2, 1, 16), ("up.A.1", 128, 2, 1, 16), ("up.A.2", 128, 2, 1, 16)]
    m = SDXLFlowMatchQLoRA(B=2, latent=32, stacks=stacks, n_ctx=20, context_dim=128, seed=5, pooled_dim=1280)
    g = torch.Generator(device=DEV).manual_seed(11)
    with torch.no_grad():  # non-zero adapters so that both LoRA factors receive gradient
        m.core.params.copy_((torch.randn(m.core.params.shape, device=DEV, generator=g) * 0.05).bfloat16())
    lat, ctx, pooled, sizes = m.make_inputs(seed=3, latent=latent)
    t = torch.tensor([0.3, 0.8], device=DEV)
    eps = rnd(*lat.shape, seed=12)
    loss, v = m.step(lat, ctx, pooled, sizes, t=t, eps=eps, optimizer_step=False)
    torch.cuda.synchronize()
    sk = {k: (getattr(m, k).w.float().cpu(), None if getattr(m, k).b is None else getattr(m, k).b.float().cpu())
          for k in ("t1", "t2", "l1", "l2", "e_in", "e_down", "e_up", "m_in", "m_down", "m_up", "m_out")}
    ws = []
    for (_, C, HW, st) in m.core.stacks:
        ws.append((_export_stack(st), st.heads, st.depth))
    rl, rv = SO.flow_match_loss(lat.cpu(), t.cpu(), eps.cpu(), ctx.float().cpu().view(2, 20, 128),
                                pooled.float().cpu(), sizes.cpu(), sk, ws, 16, 1.0)
    rl.backward()
    assert abs(loss.item() - rl.item()) < 1e-2 * rl.item()
    assert rel(v, rv.detach()) < 3e-2
    bad = []
    for (_, _, _, st), (w, _, _) in zip(m.core.stacks, ws):
        bad += _check_adapter_grads(_grad_pairs(st), w, min_cos=0.98)
    assert not bad, bad[:8]


@pytest.mark.parametrize("C,heads,depth,side,B", [(640, 10, 2, 64, 1), (1280, 20, 1, 32, 2), (640, 10, 1, (56, 72), 1),
                                                   (1280, 20, 1, (28, 36), 2), (1280, 20, 1, (44, 24), 1)])
def test_production_shape_stack_matches_oracle(C, heads, depth, side, B):
    """The benched shapes: a 640-channel SpatialTransformer (2 blocks, 64 x 64 latents) and one 1280-channel block
    at 32 x 32, context 231 x 2048, NF4 bases (w_kmajor=0 input-gradient GEMMs at N = 1280, the K = 5120 ff
    GEMM), random non-zero LoRA adapters: output, input gradient and every adapter gradient vs the fp32 oracle.
    Also the stage shapes of the 896 x 1152 bucket (56 x 72 and 28 x 36: 4032 / 1008 tokens) and of 1408 x 768
    (44 x 24 = 1056 tokens) -- token counts that are not multiples of the 64-row tiles."""
    sh, sw = (side, side) if isinstance(side, int) else side
    from vpt.sdxl_train import SDXLStacksQLoRA
    m = SDXLStacksQLoRA(B=B, stacks=[("s", C, heads, depth, sh)], n_ctx=231, context_dim=2048, seed=21)
    g = torch.Generator(device=DEV).manual_seed(22)
    with torch.no_grad():
        m.params.copy_((torch.randn(m.params.shape, device=DEV, generator=g) * 0.03).bfloat16())
    st = m.stacks[0][3]
    HW = sh * sw
    x = rnd(B, C, HW, seed=23)
    ctx = rnd(B * 231, 2048, seed=24)
    dy = rnd(B, C, HW, scale=1e-2, seed=25)
    m.grads.zero_()
    y = st.forward(x, ctx, B, HW, 231)
    dx, _ = st.backward(dy, need_dctx=False)
    torch.cuda.synchronize()
    w = _export_stack(st)
    xr = x.float().cpu().view(B, C, sh, sw).requires_grad_(True)
    yr = SO.spatial_forward(xr, ctx.float().cpu().view(B, 231, 2048), w, heads, depth, 16, 1.0)
    yr.backward(dy.float().cpu().view(B, C, sh, sw))
    assert rel(y, yr.detach().reshape(B, C, HW)) < 2e-2
    assert rel(dx, xr.grad.reshape(B, C, HW)) < 3e-2
    bad = _check_adapter_grads(_grad_pairs(st), w, min_cos=0.99)
    assert not bad, bad[:8]


def test_production_step_runs_every_bucket_with_unit_scale_loss():
    """The benched config-5 model (11 stacks, 70 blocks, 700 adapters; B=1 here) steps each of the five buckets the
    bench draws (896 x 1152 ... 1408 x 768: latents 112 x 144 ... 176 x 96) back to back on one set of buffers: the
    loss stays finite and O(1) on unit-variance targets (the calibrated skeleton: velocity MSE ~ 2-3, not hundreds),
    and the adapters move."""
    from vpt.sdxl_flow import SDXL_BUCKETS_5, SDXLFlowMatchQLoRA
    m = SDXLFlowMatchQLoRA(B=1, device=DEV, seed=0)
    p0 = m.core.params.float().clone()
    for (W, H) in SDXL_BUCKETS_5:
        lat, ctx, pooled, sizes = m.make_inputs(seed=W, latent=(H // 8, W // 8))
        loss, v = m.step(lat, ctx, pooled, sizes)
        assert v.shape == lat.shape
        lv = loss.item()
        assert math.isfinite(lv) and 0.5 < lv < 10.0, (W, H, lv)
    torch.cuda.synchronize()
    assert (m.core.params.float() - p0).abs().max().item() > 0
