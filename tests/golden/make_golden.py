"""Generates the golden fixtures in tests/golden/ by running the REFERENCE (p1atdev/vision-pt at
/root/reference) on CPU in the survey container. Only the resulting tensors are committed (no
reference source travels). Re-run: `python tests/golden/make_golden.py [sampler|sdxl]` (needs /root/reference).

Import recipe: SURVEY.md Appendix A (Recipe A for the denoiser/config/class encoder, Recipe B
stubs for train/jit/arb_class_to_image.py to reach JiTModel.image_to_velocity).

Fixtures:
  jit_micro.safetensors  micro JiT (D=192, 3 heads, depth 3, context from block 1, ctx_dim 64,
                         2 x 64x48 images, 8 context tokens, one padded) — fp32 reference forward,
                         image- and velocity-target losses, full gradients of the small
                         parameters and (norm, sum, first 64) of every parameter gradient.
  jit_micro_fuse.safetensors  the same with do_context_fuse=True (context tokens appended once at
                         context_start_block and carried through the later blocks, denoiser.py:1087-1113).
  jit_c1.safetensors     BASELINE config 1 (D=256, 4 heads, depth 2, ctx_dim 256, context in both
                         blocks, 4 x 256^2): loss, output checksums, per-parameter grad norms.
  ops.safetensors        timestep embedding (t = 0..9999 subsample + fractional), RoPE tables of
                         the 7 benchmark buckets (checksums + head/tail rows), tokenizer ids/masks,
                         bucket lists.
  sdxl_block.safetensors the reference's SDXL TransformerBlock (src/models/sdxl/denoiser.py:208-280) with
                         its 10 Linear layers wrapped by the reference LoRALinear (src/modules/peft/lora.py,
                         rank 16, alpha 8), base weights = NF4-dequantised (oracle.sdxl_oracle, restated bnb format):
                         dim 128, 2 heads, context_dim 96, 2 x 80 tokens, 20 context tokens. Forward output
                         and gradients (input, context, every LoRA weight) of sum(out * dy), once in fp32
                         with fp32 attention and once in the reference's native bf16.
  sdxl_spatial.safetensors  the reference SpatialTransformer (denoiser.py:283-365): GroupNorm(32, 128), NF4
                         proj_in / proj_out, 2 LoRA-wrapped blocks, context 128, 2 x 8x8 latents, 20 context
                         tokens; fp32 and native-bf16 forward / input, context and adapter grads of sum(out*dy).
  saving.safetensors     ModelSavingStrategy.should_save over every (epoch, step) of six strategies, which
                         invalid strategies raise, and the callback file-name template.
  timestep.safetensors   sample_timestep for the scale_shift_sigmoid / sigmoid / uniform / shift_sigmoid /
                         flux_shift samplers (two latent shapes, two global-RNG seeds, non-default kwargs).
  init.safetensors       JiT.initialize_weights + ClassEncoder.initialize_weights on the micro config: per
                         parameter the kind (normal / ones / zeros), mean, std, numel.
  ref_bf16_error.safetensors  the reference's own bf16-autocast step vs its fp32 step on the GPU parity
                         test's cases (micro, C1, JiT-B/16 256^2 B=2 and 1024^2 B=1): per-parameter gradient
                         rel-L2, prediction and loss rel (`make_golden.py bf16err`).
  sampler.safetensors    JiTModel.generate (src/models/jit/pipeline.py:378-488) on the micro config,
                         float32 execution, class context, 4 Euler steps, 2 x 64x48: starting noise,
                         token ids/masks and the final image for four cases (CFG 2.0; no CFG; CFG 3.0
                         inside cfg_time_range [0.2, 0.6]; velocity prediction). Metadata: the
                         reference JiTModel state-dict keys and shapes (checkpoint layout).
Weights are not stored: they are regenerated from oracle.jit_oracle.make_weights(cfg, seed).
"""

from __future__ import annotations

import ast
import importlib
import importlib.machinery
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
from oracle.jit_oracle import OracleConfig, make_weights  # noqa: E402
from tests.golden.golden_configs import c1_config, make_batch, micro_config, micro_fuse_config  # noqa: E402

torch.set_num_threads(8)


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)

    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__spec__ = importlib.machinery.ModuleSpec(name, None)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Any:
        def __init__(self, *a, **k):
            pass

    stub("wandb", Image=_Any)
    stub("imagesize", get=lambda p: (0, 0))
    stub("polars")
    stub("src.dataset.text_to_image", TextToImageDatasetConfig=object)
    stub("src.dataset.square_class_image", SquareClassImageDatasetConfig=object)
    stub("src.utils.grid", images_to_grid_image=None)
    bnb = stub("bitsandbytes")
    bnb.__path__ = []
    bnb.nn = stub("bitsandbytes.nn", Linear4bit=nn.Linear, Linear8bitLt=nn.Linear, Params4bit=nn.Parameter,
                  Int8Params=nn.Parameter)
    bnb.functional = stub("bitsandbytes.functional", quantize_4bit=None)
    ao = stub("torchao")
    ao.__path__ = []
    stub("torchao.float8").__path__ = []
    stub("torchao.float8.float8_linear", Float8Linear=nn.Linear)
    sys.path.insert(0, REF + "/train/jit")
    arb = importlib.import_module("arb_class_to_image")
    den = importlib.import_module("src.models.jit.denoiser")
    cfgm = importlib.import_module("src.models.jit.config")
    ce = importlib.import_module("src.models.jit.class_encoder")
    emb = importlib.import_module("src.modules.timestep.embedding")
    fm = importlib.import_module("src.modules.loss.flow_match")
    # generate_buckets is pure numpy but its module imports torchvision: exec the function source
    src = open(REF + "/src/dataset/aspect_ratio_bucket.py").read()
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "generate_buckets")
    ns = {"np": np}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "aspect_ratio_bucket.py", "exec"), ns)
    return types.SimpleNamespace(arb=arb, den=den, cfg=cfgm, ce=ce, emb=emb, fm=fm, generate_buckets=ns["generate_buckets"])


def ref_config(R, oc: OracleConfig):
    return R.cfg.DenoiserConfig(
        patch_size=oc.patch_size, hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
        bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim, context_start_block=oc.context_start_block,
        do_context_fuse=oc.do_context_fuse,
        rope_axes_dims=oc.rope_axes_dims, rope_axes_lens=oc.rope_axes_lens, rope_zero_centered=oc.rope_zero_centered)


def run_reference(R, oc: OracleConfig, weights, batch, loss_target):
    model = R.den.Denoiser(ref_config(R, oc))
    sd = {k: v for k, v in weights.items() if not k.startswith("class_encoder.")}
    model.load_state_dict(sd, strict=True)
    model.train()
    emb = weights["class_encoder.embedding.weight"].clone().requires_grad_(True)
    x = batch["image"]
    t = batch["t"]
    orig = torch.randn_like
    torch.randn_like = lambda ten, *a, **k: batch["noise"].to(ten.dtype)
    try:
        z, _ = R.fm.prepare_scaled_noised_latents(latents=x, timestep=t, noise_scale=1.0)  # flow_match.py:60-74
    finally:
        torch.randn_like = orig
    ctx = F.embedding(batch["ids"], emb, padding_idx=emb.shape[0] - 1)  # nn.Embedding(padding_idx=V)
    pred = model(image=z.float(), timestep=t.float(), context=ctx, original_size=batch["original_size"],
                 target_size=batch["target_size"], crop_coords=batch["crop_coords"], context_mask=batch["mask"])
    if loss_target == "image":
        loss = F.mse_loss(pred, x.float())  # arb_class_to_image.py:139-144
    else:
        itv = R.arb.JiTModel.image_to_velocity
        pv = itv(None, image=pred, noisy=z, timestep=t, clamp_eps=0.05)
        tv = itv(None, image=x.float(), noisy=z, timestep=t, clamp_eps=0.05)
        loss = F.mse_loss(pv, tv)  # arb_class_to_image.py:119-138
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    grads["class_encoder.embedding.weight"] = emb.grad.detach().clone()
    return loss.detach(), pred.detach(), z.detach(), grads


def grad_summary(prefix, grads, out, full_small=4096):
    for n, gr in grads.items():
        g = gr.float().reshape(-1)
        out[f"{prefix}gnorm/{n}"] = g.norm().reshape(1)
        out[f"{prefix}gsum/{n}"] = g.sum().reshape(1)
        out[f"{prefix}ghead/{n}"] = g[:64].clone()
        if g.numel() <= full_small:
            out[f"{prefix}gfull/{n}"] = g.clone()


def sampler_fixture(R, meta):
    """Runs the reference's own JiTModel.generate; the PIL conversion is swapped for the raw tensor."""
    pipe = importlib.import_module("src.models.jit.pipeline")
    oc = micro_config()
    V = 20
    w = make_weights(oc, seed=1, n_classes=V)
    l2i = os.path.join("/tmp", "vpt_golden_label2id.json")
    json.dump({f"c{i}": i for i in range(V)}, open(l2i, "w"))
    prompts = ["c1 c3", "c5 c7 c2"]
    out = {}
    keys = None
    cases = {"cfg2": dict(cfg_scale=2.0), "nocfg": dict(cfg_scale=1.0),
             "cfg3_window": dict(cfg_scale=3.0, cfg_time_range=[0.2, 0.6]), "vel_cfg2": dict(cfg_scale=2.0)}
    for name, kw in cases.items():
        cfg = R.cfg.JiTConfig(context_encoder=R.cfg.ClassContextConfig(label2id_map_path=l2i),
                              denoiser=ref_config(R, oc), model_pred="velocity" if name.startswith("vel") else "image")
        model = pipe.JiTModel(cfg)
        model.denoiser.load_state_dict({k: v for k, v in w.items() if not k.startswith("class_encoder.")}, strict=True)
        with torch.no_grad():
            model.class_encoder.embedding.weight.copy_(w["class_encoder.embedding.weight"])
        model.eval()
        model.to_pil_images = lambda t: t.clone()
        model.progress_bar = lambda total: __import__("contextlib").nullcontext(types.SimpleNamespace(update=lambda: None))
        img = model.generate(prompts, width=48, height=64, num_inference_steps=4, max_token_length=8, seed=7,
                             execution_dtype=torch.float32, device="cpu", **kw)
        out[f"{name}/image"] = img
        if keys is None:
            keys = {k: list(v.shape) for k, v in model.state_dict().items()}
    g = torch.Generator(device="cpu").manual_seed(7)
    out["noise"] = torch.randn((2, 3, 64, 48), dtype=torch.float32, generator=g)  # pipeline.py:133-140
    tok = model.class_encoder.tokenizer
    o = tok.tokenize(prompts, max_length=8)
    out["pos_ids"], out["pos_mask"] = o.class_ids, o.attention_mask
    o = tok.tokenize([""] * 2, max_length=8)
    out["neg_ids"], out["neg_mask"] = o.class_ids, o.attention_mask
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "sampler.safetensors"),
              metadata=dict(meta, prompts=json.dumps(prompts), state_dict=json.dumps(keys), cases=json.dumps(
                  {k: {kk: vv for kk, vv in v.items()} for k, v in cases.items()})))


def sdxl_block_fixture(meta):
    """Reference SDXL TransformerBlock + LoRALinear (Recipe A, sdxl variant)."""
    import functools
    from oracle import sdxl_oracle as SO

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        m = importlib.util.module_from_spec(spec)
        sys.modules[name] = m
        spec.loader.exec_module(m)
        return m

    pkg = types.ModuleType("src.models.sdxl")
    pkg.__path__ = [REF + "/src/models/sdxl"]
    sys.modules["src.models.sdxl"] = pkg
    load("src.models.sdxl.config", REF + "/src/models/sdxl/config.py")
    den = load("src.models.sdxl.denoiser", REF + "/src/models/sdxl/denoiser.py")
    lora = importlib.import_module("src.modules.peft.lora")
    dim, heads, cdim, rank, alpha, B, n, nc = 128, 2, 96, 16, 8.0, 2, 80, 20
    w = SO.make_block_weights(dim, heads, cdim, rank, seed=11)
    nf4 = {}
    for t in SO.LORA_TARGETS:
        st = SO.nf4_quantize(w[f"{t}.linear.weight"])
        nf4[t] = st
        w[f"{t}.linear.weight"] = SO.nf4_dequantize(st)
    g = torch.Generator().manual_seed(12)
    x = torch.randn(B, n, dim, generator=g)
    ctx = torch.randn(B, nc, cdim, generator=g)
    dy = torch.randn(B, n, dim, generator=g)
    out = {"x": x, "ctx": ctx, "dy": dy}
    for t, st in nf4.items():
        for k, v in st.items():
            out[f"nf4/{t}/{k}"] = v
    orig_sdpa = den.scaled_dot_product_attention
    for mode in ("fp32", "bf16"):
        dt = torch.float32 if mode == "fp32" else torch.bfloat16
        blk = den.TransformerBlock(hidden_dim=dim, num_heads=heads, head_dim=64, context_dim=cdim)
        for t in SO.LORA_TARGETS:
            parent_path, last = t.rsplit(".", 1)
            parent = blk.get_submodule(parent_path)
            wrapped = lora.LoRALinear(lora.LoRAConfig(rank=rank, alpha=alpha, dtype="float32"),
                                      parent.get_submodule(last))
            setattr(parent, last, wrapped)
        sd = blk.state_dict()
        for k in list(sd):
            if k.endswith(".alpha"):
                continue
            sd[k] = w[k].clone()
        blk.load_state_dict(sd, strict=True)
        blk = blk.to(dt)
        if mode == "fp32":  # the reference casts fp32 q/k/v to bf16 inside SDPA (attention.py:113-118)
            den.scaled_dot_product_attention = functools.partial(orig_sdpa, attention_dtype=torch.float32)
        try:
            xi = x.detach().clone().to(dt).requires_grad_(True)
            ci = ctx.detach().clone().to(dt).requires_grad_(True)
            y = blk(xi, context=ci, time_embedding=None)
            (y.float() * dy).sum().backward()
        finally:
            den.scaled_dot_product_attention = orig_sdpa
        out[f"{mode}/out"] = y.detach().float()
        out[f"{mode}/dx"] = xi.grad.float()
        out[f"{mode}/dctx"] = ci.grad.float()
        for nme, prm in blk.named_parameters():
            if "lora_" in nme and prm.grad is not None:
                out[f"{mode}/grad/{nme}"] = prm.grad.float()
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "sdxl_block.safetensors"),
              metadata=dict(meta, dims=json.dumps(dict(dim=dim, heads=heads, context_dim=cdim, rank=rank, alpha=alpha,
                                                       B=B, n=n, nc=nc, weight_seed=11))))


def sdxl_spatial_fixture(meta):
    """Reference SpatialTransformer (src/models/sdxl/denoiser.py:283-365) with 2 LoRA-wrapped blocks; every
    Linear base (proj_in / proj_out and the 20 block targets) NF4-quantised (oracle restatement) and
    dequantised, GroupNorm(32, 128); fp32 (fp32 SDPA) and native bf16 runs of sum(out * dy)."""
    import functools
    from oracle import sdxl_oracle as SO

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        m = importlib.util.module_from_spec(spec)
        sys.modules[name] = m
        spec.loader.exec_module(m)
        return m

    pkg = types.ModuleType("src.models.sdxl")
    pkg.__path__ = [REF + "/src/models/sdxl"]
    sys.modules["src.models.sdxl"] = pkg
    load("src.models.sdxl.config", REF + "/src/models/sdxl/config.py")
    den = load("src.models.sdxl.denoiser", REF + "/src/models/sdxl/denoiser.py")
    lora = importlib.import_module("src.modules.peft.lora")
    C, heads, depth, cdim, rank, alpha, B, H, W, nc = 128, 2, 2, 128, 16, 8.0, 2, 8, 8, 20
    w = SO.make_spatial_weights(C, heads, depth, cdim, rank, seed=21)
    nf4 = {}
    for k in list(w):
        if k.endswith(".linear.weight") or k in ("proj_in.weight", "proj_out.weight"):
            st = SO.nf4_quantize(w[k])
            nf4[k] = st
            w[k] = SO.nf4_dequantize(st)
    g = torch.Generator().manual_seed(22)
    x = torch.randn(B, C, H, W, generator=g)
    ctx = torch.randn(B, nc, cdim, generator=g)
    dy = torch.randn(B, C, H, W, generator=g)
    out = {"x": x, "ctx": ctx, "dy": dy}
    for k, st in nf4.items():
        for kk, v in st.items():
            out[f"nf4/{k}/{kk}"] = v
    orig_sdpa = den.scaled_dot_product_attention
    for mode in ("fp32", "bf16"):
        dt = torch.float32 if mode == "fp32" else torch.bfloat16
        st_mod = den.SpatialTransformer(in_channels=C, num_heads=heads, head_dim=64, context_dims=[cdim] * depth)
        for blk in st_mod.transformer_blocks:
            for t in SO.LORA_TARGETS:
                parent_path, last = t.rsplit(".", 1)
                parent = blk.get_submodule(parent_path)
                wrapped = lora.LoRALinear(lora.LoRAConfig(rank=rank, alpha=alpha, dtype="float32"),
                                          parent.get_submodule(last))
                setattr(parent, last, wrapped)
        sd = st_mod.state_dict()
        for k in list(sd):
            if k.endswith(".alpha"):
                continue
            sd[k] = w[k].clone()
        st_mod.load_state_dict(sd, strict=True)
        st_mod = st_mod.to(dt)
        if mode == "fp32":
            den.scaled_dot_product_attention = functools.partial(orig_sdpa, attention_dtype=torch.float32)
        try:
            xi = x.detach().clone().to(dt).requires_grad_(True)
            ci = ctx.detach().clone().to(dt).requires_grad_(True)
            y = st_mod(xi, context=ci)
            (y.float() * dy).sum().backward()
        finally:
            den.scaled_dot_product_attention = orig_sdpa
        out[f"{mode}/out"] = y.detach().float()
        out[f"{mode}/dx"] = xi.grad.float()
        out[f"{mode}/dctx"] = ci.grad.float()
        for nme, prm in st_mod.named_parameters():
            if prm.grad is not None and "lora_" in nme:
                out[f"{mode}/grad/{nme}"] = prm.grad.float()
    # the restated forward reproduces the reference's fp32 output (oracle self-check, recorded)
    ref = SO.spatial_forward(x, ctx, w, heads, depth, rank, alpha)
    out["oracle/out"] = ref.detach().float()
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "sdxl_spatial.safetensors"),
              metadata=dict(meta, dims=json.dumps(dict(C=C, heads=heads, depth=depth, context_dim=cdim, rank=rank,
                                                       alpha=alpha, B=B, H=H, W=W, nc=nc, weight_seed=21))))


def saving_fixture(meta):
    """ModelSavingStrategy.should_save (src/saving/util.py:15-120) decisions over every (epoch, step) of
    several strategies, and the callback file-name template (util.py:135, common.py:162-164)."""
    util = importlib.import_module("src.saving.util")
    cases = [dict(total_epochs=3, steps_per_epoch=10, per_epochs=1, per_steps=None, save_last=True),
             dict(total_epochs=4, steps_per_epoch=7, per_epochs=2, per_steps=None, save_last=True),
             dict(total_epochs=2, steps_per_epoch=12, per_epochs=0.25, per_steps=None, save_last=True),
             dict(total_epochs=3, steps_per_epoch=10, per_epochs=None, per_steps=4, save_last=False),
             dict(total_epochs=3, steps_per_epoch=10, per_epochs=1, per_steps=7, save_last=True),
             dict(total_epochs=2, steps_per_epoch=5, per_epochs=None, per_steps=None, save_last=False)]
    out = {}
    for ci, c in enumerate(cases):
        st = util.ModelSavingStrategy(**c)
        rows = []
        step = 0
        for epoch in range(1, c["total_epochs"] + 1):
            for _ in range(c["steps_per_epoch"]):
                step += 1
                rows.append([epoch, step, int(st.should_save(epoch, step))])
        out[f"case{ci}"] = torch.tensor(rows, dtype=torch.int64)
    bad = [dict(total_epochs=3, steps_per_epoch=10, per_epochs=1.5, per_steps=None, save_last=True),
           dict(total_epochs=3, steps_per_epoch=10, per_epochs=0.5, per_steps=3, save_last=True),
           dict(total_epochs=3, steps_per_epoch=10, per_epochs=4, per_steps=None, save_last=True),
           dict(total_epochs=3, steps_per_epoch=10, per_epochs=None, per_steps=31, save_last=True)]
    raised = []
    for c in bad:
        try:
            util.ModelSavingStrategy(**c)
            raised.append(0)
        except ValueError:
            raised.append(1)
    out["bad_raises"] = torch.tensor(raised)
    tmpl = util.ModelSavingCallback.save_name_template
    names = [tmpl.format(name="jit", epoch=e, steps=s) for e, s in ((1, 10), (12, 123456))]
    save_file(out, os.path.join(HERE, "saving.safetensors"),
              metadata=dict(meta, cases=json.dumps(cases), bad=json.dumps(bad), names=json.dumps(names),
                            template=tmpl))


def timestep_fixture(meta):
    """sample_timestep (src/modules/timestep/sampling.py:170-187) for every sampler type the JiT / SDXL
    flow-match steps select, drawn from the global RNG after torch.manual_seed(seed) on CPU."""
    samp = importlib.import_module("src.modules.timestep.sampling")
    cases = {"scale_shift_sigmoid": {}, "scale_shift_sigmoid_m0s1": {"mean": 0.0, "std": 1.0}, "sigmoid": {},
             "uniform": {}, "shift_sigmoid": {}, "flux_shift": {}, "shift_sigmoid_s2": {"sigmoid_scale": 2.0}}
    out = {}
    for name, kw in cases.items():
        typ = name.split("_m0")[0].split("_s2")[0]
        for shape in ((16, 3, 256, 256), (8, 4, 128, 96)):
            for seed in (0, 7):
                torch.manual_seed(seed)
                t = samp.sample_timestep(latents_shape=torch.Size(shape), device="cpu", sampling_type=typ, **kw)
                out[f"{name}/{'x'.join(map(str, shape))}/{seed}"] = t.float().contiguous()
    save_file(out, os.path.join(HERE, "timestep.safetensors"),
              metadata=dict(meta, cases=json.dumps({k: v for k, v in cases.items()})))


def init_fixture(R, meta):
    """JiT.initialize_weights (src/models/jit/denoiser.py:764-798) + ClassEncoder.initialize_weights
    (class_encoder.py:124-125) on the micro config: per parameter [kind (0 normal / 1 ones / 2 zeros), mean,
    std, numel] -- the distribution each tensor is drawn from (the RNG stream itself is not part of the API)."""
    oc = micro_config()
    torch.manual_seed(0)
    model = R.den.Denoiser(ref_config(R, oc))
    model.initialize_weights()
    enc = R.ce.ClassEncoder(label2id={f"c{i}": i for i in range(20)}, embedding_dim=oc.context_dim)
    enc.initialize_weights()
    named = dict(model.named_parameters())
    named["class_encoder.embedding.weight"] = enc.embedding.weight
    names = sorted(named)
    rows = []
    for n in names:
        t = named[n].detach().double()
        kind = 1 if bool((t == 1).all()) else 2 if bool((t == 0).all()) else 0
        rows.append([kind, t.mean().item(), t.std().item() if t.numel() > 1 else 0.0, t.numel()])
    save_file({"stats": torch.tensor(rows, dtype=torch.float64)}, os.path.join(HERE, "init.safetensors"),
              metadata=dict(meta, names=json.dumps(names)))


def run_reference_bf16(R, oc: OracleConfig, weights, batch, loss_target):
    """The reference as its trainer runs it (SURVEY gotcha #5): bf16 weights, forward and backward under
    bf16 autocast (accelerate mixed_precision=bf16, src/trainer/common.py:322), fp16 images, fp32 loss."""
    model = R.den.Denoiser(ref_config(R, oc))
    sd = {k: v for k, v in weights.items() if not k.startswith("class_encoder.")}
    model.load_state_dict(sd, strict=True)
    model = model.to(torch.bfloat16)
    model.train()
    emb = weights["class_encoder.embedding.weight"].clone().to(torch.bfloat16).requires_grad_(True)
    x, t = batch["image"], batch["t"]
    orig = torch.randn_like
    torch.randn_like = lambda ten, *a, **k: batch["noise"].to(ten.dtype)
    try:
        z, _ = R.fm.prepare_scaled_noised_latents(latents=x, timestep=t, noise_scale=1.0)
    finally:
        torch.randn_like = orig
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ctx = F.embedding(batch["ids"], emb, padding_idx=emb.shape[0] - 1)
        pred = model(image=z, timestep=t.to(torch.bfloat16), context=ctx, original_size=batch["original_size"],
                     target_size=batch["target_size"], crop_coords=batch["crop_coords"], context_mask=batch["mask"])
        assert loss_target == "image"
        loss = F.mse_loss(pred, x)
    loss.backward()
    grads = {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}
    grads["class_encoder.embedding.weight"] = emb.grad.detach().float().clone()
    return loss.detach().float(), pred.detach().float(), grads


def bf16_error_fixture(R, meta):
    """How far the REFERENCE's own bf16-autocast training step is from its fp32 step, per parameter gradient
    (whole-tensor rel-L2), prediction and loss -- on the exact cases tests/test_parity_gpu.py runs. The GPU
    parity test holds the HIP step to SURVEY §8(c)'s bar, except on a parameter where the reference's own bf16
    step is already further than that bar from fp32."""
    from oracle.jit_oracle import jit_b16
    cases = {"micro": (micro_config(), 20, 1, dict(B=2, H=64, W=48, n_ctx=8, seed=2)),
             "c1": (c1_config(), 1000, 3, dict(B=4, H=256, W=256, n_ctx=64, seed=4, padded_rows=(1, 3))),
             "jitb16-256x256-B2": (jit_b16(), 1000, 11, dict(B=2, H=256, W=256, n_ctx=64, seed=12)),
             "jitb16-1024x1024-B1": (jit_b16(), 1000, 11, dict(B=1, H=1024, W=1024, n_ctx=64, seed=12))}
    # every other GPU parity case the CPU's memory holds (B = 8 at 1024^2 does not: the parity test bounds it
    # with the largest per-parameter entry over the five 1024^2 B = 2 buckets)
    for (H, W, B) in [(1024, 1024, 2), (1088, 960, 2), (960, 1088, 2), (896, 1152, 2), (1152, 896, 2), (512, 512, 16)]:
        cases[f"jitb16-{W}x{H}-B{B}"] = (jit_b16(), 1000, 11, dict(B=B, H=H, W=W, n_ctx=64, seed=12))
    only = os.environ.get("BF16ERR_CASES")
    if only:
        cases = {k: v for k, v in cases.items() if k in only.split(",")}
    path = os.path.join(HERE, "ref_bf16_error.safetensors")
    out, names = {}, {}
    if os.path.exists(path):  # incremental: keep the cases already computed
        from safetensors import safe_open
        from safetensors.torch import load_file
        with safe_open(path, "pt") as f:
            names = json.loads(f.metadata()["names"])
        out = dict(load_file(path))
    for case, (oc, V, wseed, bk) in cases.items():
        if case in names:
            continue
        w = make_weights(oc, seed=wseed, n_classes=V)
        kw = {k: v for k, v in bk.items() if k not in ("B", "H", "W", "n_ctx", "seed")}
        batch = make_batch(oc, bk["B"], bk["H"], bk["W"], bk["n_ctx"], V, seed=bk["seed"], **kw)
        l32, p32, _, g32 = run_reference(R, oc, w, batch, "image")
        l16, p16, g16 = run_reference_bf16(R, oc, w, batch, "image")
        order = sorted(g32)
        names[case] = order
        rels = [((g16[n] - g32[n].float()).norm() / g32[n].float().norm().clamp_min(1e-30)).item() for n in order]
        out[f"{case}/grad_rel"] = torch.tensor(rels, dtype=torch.float64)
        out[f"{case}/pred_rel"] = ((p16 - p32).norm() / p32.norm()).double().reshape(1)
        out[f"{case}/loss_rel"] = ((l16 - l32).abs() / l32).double().reshape(1)
        print(case, "pred", out[f"{case}/pred_rel"].item(), "loss", out[f"{case}/loss_rel"].item(),
              "worst grad", max(zip(rels, order)), flush=True)
        save_file(out, path, metadata=dict(meta, names=json.dumps(names)))


def micro_fixture(R, meta, oc: OracleConfig, name: str):
    """jit_micro (context appended before every block from context_start_block and stripped after it) and
    jit_micro_fuse (do_context_fuse=True: appended once at context_start_block and carried to the end,
    denoiser.py:1087-1113): both loss targets, the same weights and batch."""
    V = 20
    w = make_weights(oc, seed=1, n_classes=V)
    batch = make_batch(oc, 2, 64, 48, 8, V, seed=2)
    out = {k: v for k, v in batch.items()}
    for lt in ("image", "velocity"):
        loss, pred, z, grads = run_reference(R, oc, w, batch, lt)
        out[f"{lt}/loss"] = loss.reshape(1)
        out[f"{lt}/pred"] = pred
        grad_summary(f"{lt}/", grads, out)
    out["z"] = z
    out["wsum"] = torch.stack([w[k].double().sum().float() for k in sorted(w)])
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, name + ".safetensors"),
              metadata=dict(meta, do_context_fuse=str(oc.do_context_fuse)))


def objectives_fixture(R, meta):
    """jit_objectives: the reference's OWN train_step functions, run with a stand-in `self` (the trainer's
    accelerator / logging plumbing replaced; t and the noise draw taken from the batch):
      vpred    -- train/jit/class_to_image.py:166-243 with model_pred="velocity" (treat_loss :146-156: target
                  clean - noise, no clamp), the micro batch of jit_micro;
      lowres_x -- train/jit/arb_class_to_image.py:153-276 with loss_target "image" and lowres_loss [0.5, 0.25]
                  (two extra passes on F.interpolate(mode="area") inputs, arb:228-272), a 2 x 128 x 64 batch;
      lowres_v -- the same with loss_target "velocity" and lowres_loss [0.5]."""
    import functools
    cti = importlib.import_module("class_to_image")
    oc = micro_config()
    V = 20
    w = make_weights(oc, seed=1, n_classes=V)
    out = {}
    cases = {"vpred": (cti, "velocity", "velocity", [], make_batch(oc, 2, 64, 48, 8, V, seed=2)),
             "lowres_x": (R.arb, "image", "image", [0.5, 0.25], make_batch(oc, 2, 128, 64, 8, V, seed=5)),
             "lowres_v": (R.arb, "image", "velocity", [0.5], make_batch(oc, 2, 128, 64, 8, V, seed=5))}
    def run(mod, model_pred, loss_target, lowres, batch, bf16):
        """The reference's train_step on `batch`: fp32, or as its trainer runs it (bf16 weights, forward and
        backward under bf16 autocast, fp16 images; run_reference_bf16's convention)."""
        dt = torch.bfloat16 if bf16 else torch.float32
        den = R.den.Denoiser(ref_config(R, oc))
        den.load_state_dict({k: v for k, v in w.items() if not k.startswith("class_encoder.")}, strict=True)
        den = den.to(dt)
        den.train()
        emb = w["class_encoder.embedding.weight"].clone().to(dt).requires_grad_(True)
        preds = []

        def denoiser(**kw):
            o = den(**kw)
            preds.append(o.detach().float().clone())
            return o

        class ClassEnc:
            @staticmethod
            def encode_prompts(caption, max_token_length):
                return F.embedding(batch["ids"], emb, padding_idx=emb.shape[0] - 1), batch["mask"]

        mcfg = types.SimpleNamespace(torch_dtype=dt, drop_context_rate=0.0, train_class_encoder=True,
                                     max_token_length=batch["ids"].shape[1], timestep_sampling="scale_shift_sigmoid",
                                     noise_scale=1.0, timestep_eps=0.05, model_pred=model_pred,
                                     loss_target=loss_target, lowres_loss=lowres)
        model = types.SimpleNamespace(text_encoder=None, class_encoder=ClassEnc(), denoiser=denoiser,
                                      image_to_velocity=functools.partial(mod.JiTModel.image_to_velocity, None))
        me = types.SimpleNamespace(model_config=mcfg, model=model, accelerator=types.SimpleNamespace(device="cpu"),
                                   log=lambda *a, **k: None)
        me.treat_loss = functools.partial(mod.JiTForClassToImageTraining.treat_loss, me)
        # the fp32 reference run (as every fixture here): the fp16 image / noise values as f32 tensors (with fp16 tensors
        # the velocity target's mixed-dtype mse_loss has no CPU backward outside autocast); the bf16 run: fp16 images
        rb = {"image": batch["image"] if bf16 else batch["image"].float(), "caption": [""] * batch["image"].shape[0],
              "original_size": batch["original_size"], "target_size": batch["target_size"],
              "crop_coords_top_left": batch["crop_coords"]}
        old_st, old_rl = mod.sample_timestep, torch.randn_like
        mod.sample_timestep = lambda **kw: batch["t"]
        torch.randn_like = lambda ten, *a, **k: batch["noise"].to(ten.dtype)
        try:
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
                loss = mod.JiTForClassToImageTraining.train_step(me, rb)
        finally:
            mod.sample_timestep, torch.randn_like = old_st, old_rl
        loss.backward()
        assert len(preds) == 1 + len(lowres)
        grads = {n: p.grad.detach().float().clone() for n, p in den.named_parameters()}
        grads["class_encoder.embedding.weight"] = emb.grad.detach().float().clone()
        return loss.detach().float(), preds[0], grads

    names = {}
    for case, (mod, model_pred, loss_target, lowres, batch) in cases.items():
        loss, pred, grads = run(mod, model_pred, loss_target, lowres, batch, False)
        _, _, g16 = run(mod, model_pred, loss_target, lowres, batch, True)
        for k in ("image", "noise", "t", "ids", "mask", "original_size", "target_size", "crop_coords"):
            out[f"{case}/in/{k}"] = batch[k]
        out[f"{case}/loss"] = loss.reshape(1)
        out[f"{case}/pred"] = pred
        grad_summary(f"{case}/", grads, out)
        # the reference's own bf16-vs-fp32 gradient error on this case (the parity bars' yardstick, as ref_bf16_error)
        names[case] = sorted(grads)
        out[f"{case}/bf16_grad_rel"] = torch.tensor(
            [((g16[n] - grads[n]).norm() / grads[n].norm().clamp_min(1e-30)).item() for n in names[case]],
            dtype=torch.float64)
        print(case, loss.item(), "worst bf16 rel", out[f"{case}/bf16_grad_rel"].max().item(), flush=True)
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "jit_objectives.safetensors"),
              metadata=dict(meta, lowres=json.dumps({c: v[3] for c, v in cases.items()}), names=json.dumps(names)))


def main():
    R = import_reference()
    meta = {"torch": torch.__version__, "threads": str(torch.get_num_threads()), "reference": REF}
    if len(sys.argv) > 1 and sys.argv[1] == "bf16err":
        bf16_error_fixture(R, meta)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "sampler":
        sampler_fixture(R, meta)
        print("sampler", os.path.getsize(os.path.join(HERE, "sampler.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "sdxl_spatial":
        sdxl_spatial_fixture(meta)
        print("sdxl_spatial", os.path.getsize(os.path.join(HERE, "sdxl_spatial.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "saving":
        saving_fixture(meta)
        print("saving", os.path.getsize(os.path.join(HERE, "saving.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "init":
        init_fixture(R, meta)
        print("init", os.path.getsize(os.path.join(HERE, "init.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "timestep":
        timestep_fixture(meta)
        print("timestep", os.path.getsize(os.path.join(HERE, "timestep.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "objectives":
        objectives_fixture(R, meta)
        print("jit_objectives", os.path.getsize(os.path.join(HERE, "jit_objectives.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "fuse":
        micro_fixture(R, meta, micro_fuse_config(), "jit_micro_fuse")
        print("jit_micro_fuse", os.path.getsize(os.path.join(HERE, "jit_micro_fuse.safetensors")))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "sdxl":
        sdxl_block_fixture(meta)
        print("sdxl_block", os.path.getsize(os.path.join(HERE, "sdxl_block.safetensors")))
        return

    # ---------------- micro
    micro_fixture(R, meta, micro_config(), "jit_micro")
    micro_fixture(R, meta, micro_fuse_config(), "jit_micro_fuse")

    # ---------------- C1 tiny (BASELINE config 1)
    oc = c1_config()
    V = 1000
    w = make_weights(oc, seed=3, n_classes=V)
    batch = make_batch(oc, 4, 256, 256, 64, V, seed=4, padded_rows=(1, 3))
    loss, pred, z, grads = run_reference(R, oc, w, batch, "image")
    out = {"loss": loss.reshape(1), "pred_sum": pred.double().sum().float().reshape(1),
           "pred_sq": pred.double().pow(2).sum().float().reshape(1), "pred_head": pred.reshape(-1)[:256].clone(),
           "pred_tail": pred.reshape(-1)[-256:].clone()}
    gsum = {}
    grad_summary("", grads, gsum, full_small=0)
    out.update({k: v for k, v in gsum.items() if not k.startswith("ghead")})
    save_file({k: v.contiguous() for k, v in out.items()}, os.path.join(HERE, "jit_c1.safetensors"), metadata=meta)

    # ---------------- per-op vectors
    ops = {}
    tt = torch.cat([torch.arange(0, 10000, 37).float(), torch.tensor([0.5, 0.123, 0.999, 1024.0, 2048.0])])
    ops["temb/t"] = tt
    ops["temb/out"] = R.emb.get_timestep_embedding(tt, 256, flip_sin_to_cos=True, downscale_freq_shift=0)
    cfgB = R.cfg.JiT_B_16_Config()
    model_b = None
    rope = R.den.RopeEmbedder(rope_theta=cfgB.rope_theta, axes_dims=cfgB.rope_axes_dims,
                              axes_lens=cfgB.rope_axes_lens, zero_centered=cfgB.rope_zero_centered)
    for (Wd, Hd) in [(256, 256), (512, 512), (1024, 1024), (960, 1088), (1088, 960), (896, 1152), (1152, 896)]:
        ids = [rope.prepare_image_position_ids(Hd, Wd, 16, 3), rope.prepare_context_position_ids(6, 2),
               rope.prepare_context_position_ids(4, 1), rope.prepare_context_position_ids(64, 0)]
        fc = torch.cat([rope(position_ids=i.unsqueeze(0)) for i in ids], 1)[0]  # denoiser.py:1032-1051
        key = f"rope/{Wd}x{Hd}"
        ops[key + "/cos_sum"] = fc.real.double().sum().float().reshape(1)
        ops[key + "/sin_sum"] = fc.imag.double().sum().float().reshape(1)
        ops[key + "/head"] = torch.view_as_real(fc[:8]).contiguous()
        ops[key + "/tail"] = torch.view_as_real(fc[-80:]).contiguous()
        ops[key + "/n"] = torch.tensor([fc.shape[0]])
    # tokenizer
    label2id = {f"tag{i}": i for i in range(12)}
    tok = R.ce.ClassTokenizer(label2id=label2id, splitter=" ", do_mask_padding=True)
    caps = ["tag1 tag3 tag3", "", "tag11 unknown tag0", " ".join(f"tag{i % 12}" for i in range(20))]
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        o = tok.tokenize(caps, max_length=8)
    ops["tok/ids"] = o.class_ids
    ops["tok/mask"] = o.attention_mask
    meta_ops = dict(meta, captions=json.dumps(caps), label2id=json.dumps(label2id))
    for args in [(1024 ** 2, 1024, 64, 64), (64 ** 2, 64, 64, 64), (1024 ** 2, 1024, 64, 384), (256 ** 2, 256, 128, 256)]:
        b = R.generate_buckets(*args)
        ops["buckets/" + "_".join(map(str, args))] = torch.from_numpy(np.asarray(b, dtype=np.int64))
    # one rms_norm + apply_rope vector (denoiser.py:98-111, norm.py:20-27)
    g = torch.Generator().manual_seed(5)
    xq = torch.randn(2, 3, 10, 64, generator=g)
    fc = torch.polar(torch.ones(10, 32), torch.rand(10, 32, generator=g) * 6)
    ops["rope_apply/x"] = xq
    ops["rope_apply/freqs"] = torch.view_as_real(fc).contiguous()
    ops["rope_apply/out"] = R.den.apply_rope(xq, fc.unsqueeze(0).repeat(2, 1, 1))
    nw = torch.randn(64, generator=g)
    norm = R.den.get_norm_layer("rms", 64, eps=1e-6)
    with torch.no_grad():
        norm.weight.copy_(nw)
    ops["rms/w"] = nw
    ops["rms/out"] = norm(xq).detach()
    save_file({k: v.contiguous() for k, v in ops.items()}, os.path.join(HERE, "ops.safetensors"), metadata=meta_ops)
    sampler_fixture(R, meta)
    sdxl_block_fixture(meta)
    timestep_fixture(meta)
    init_fixture(R, meta)
    sdxl_spatial_fixture(meta)
    saving_fixture(meta)
    for f in ("jit_micro", "jit_micro_fuse", "jit_c1", "ops", "sampler", "sdxl_block", "timestep", "init", "sdxl_spatial", "saving"):
        print(f, os.path.getsize(os.path.join(HERE, f + ".safetensors")))


if __name__ == "__main__":
    main()
