"""a26 on the GPU: the training loop (vpt.trainer.JiTTrainLoop) over a micro JiT config -- optimizer
train()/eval() toggles, gradient accumulation (micro-step gradients add up in the flat f32 buffer), the
reference's checkpoint names incl. the EMA copy, and the EMA kernel against the reference's bf16 arithmetic
(torch.optim.swa_utils.get_ema_avg_fn on bf16 tensors)."""
import os

import pytest
import torch
from safetensors.torch import load_file

from tests.golden import golden_configs as GC

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(seed=1):
    from vpt.config import DenoiserConfig, JiTTrainingConfig
    from vpt.jit_train import ClassTokenizer, JiTTrainer
    oc = GC.micro_config()
    cfg = DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                         bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                         context_start_block=oc.context_start_block)
    tr = JiTTrainer(cfg, 20, JiTTrainingConfig(loss_target="image", drop_context_rate=0.0), device=DEV, seed=seed)
    tr.engine.init_weights(seed=0)
    tok = ClassTokenizer({f"c{i}": i for i in range(20)})
    g = torch.Generator().manual_seed(seed)
    batches = []
    for k in range(4):
        img = (torch.rand(2, 3, 64, 48, generator=g) * 2 - 1).half().to(DEV)
        size = torch.tensor([[64, 48]] * 2, device=DEV)
        batches.append(dict(image=img, caption=[f"c{k} c{k + 3}", f"c{2 * k}"], original_size=size,
                            target_size=size.clone(), crop_coords_top_left=torch.zeros(2, 2, dtype=torch.long,
                                                                                        device=DEV)))
    return tr, tok, batches


def test_gradient_accumulation_adds_micro_step_gradients():
    tr, tok, bs = _setup()
    g = torch.Generator().manual_seed(5)
    noise = [torch.randn(2, 3, 64, 48, generator=g).half().to(DEV) for _ in range(2)]  # same eps both passes
    grads = []
    for b, nz in zip(bs[:2], noise):
        ids, mask = tok.tokenize(b["caption"], max_length=8)
        tr.step(b["image"], ids, mask, b["original_size"], b["target_size"], b["crop_coords_top_left"],
                t=torch.tensor([0.4, 0.7]), noise=nz, drop_context=False)
        grads.append(tr.engine.grads.clone())
    for i, (b, nz) in enumerate(zip(bs[:2], noise)):
        ids, mask = tok.tokenize(b["caption"], max_length=8)
        tr.step(b["image"], ids, mask, b["original_size"], b["target_size"], b["crop_coords_top_left"],
                t=torch.tensor([0.4, 0.7]), noise=nz, drop_context=False, accumulate=i > 0)
    torch.cuda.synchronize()
    ref = grads[0] + grads[1]
    assert ((tr.engine.grads - ref).norm() / ref.norm()).item() < 1e-6


def test_train_loop_saving_ema_and_optimizer_modes(tmp_path):
    from vpt.optim import RAdamScheduleFreeFlat
    from vpt.trainer import JiTTrainLoop, SafetensorsSaver, SavingStrategy
    tr, tok, bs = _setup(seed=2)
    opt = RAdamScheduleFreeFlat(tr.engine.params, tr.engine.grads, lr=1e-3)
    loop = JiTTrainLoop(tr, opt, bs, tok, num_train_epochs=2, gradient_accumulation_steps=2,
                        saving=SavingStrategy(2, len(bs), per_epochs=None, per_steps=4),
                        savers=[SafetensorsSaver("jit", str(tmp_path))], use_ema=True, ema_decay=0.9,
                        max_token_length=8)
    steps = loop.train()
    torch.cuda.synchronize()
    assert steps == 8 and opt.param_groups[0]["k"] == 4 and not opt.param_groups[0]["train_mode"]
    assert all(l == l for l in loop.losses) and len(loop.losses) == 8
    names = sorted(os.listdir(tmp_path))
    assert names == ["ema_jit_00001e_000004s.safetensors", "ema_jit_00002e_000008s.safetensors",
                     "jit_00001e_000004s.safetensors", "jit_00002e_000008s.safetensors"]
    sd = load_file(os.path.join(tmp_path, names[-1]))
    assert "class_encoder.embedding.weight" in sd and any(k.startswith("denoiser.") for k in sd)
    assert loop.ema.n_averaged == 4


@pytest.mark.parametrize("decay", [0.9, 0.9999])
def test_ema_kernel_matches_bf16_reference_arithmetic(decay):
    """0.9999 is the reference default (src/config.py ema_decay): torch rounds the Python double 1 - decay."""
    from vpt import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    p = torch.randn(100003, device=DEV, generator=g).bfloat16()
    ema = torch.empty_like(p)
    ops.ema_update(ema, p, decay, True)
    assert torch.equal(ema, p)
    ref = ema.clone()
    for _ in range(3):
        p = (p.float() + 0.1 * torch.randn(p.shape, device=DEV, generator=g)).bfloat16()
        ops.ema_update(ema, p, decay, False)
        ref = decay * ref + (1 - decay) * p  # get_ema_avg_fn on bf16 tensors (swa_utils)
    torch.cuda.synchronize()
    assert torch.equal(ema, ref)
    # a 1-element offset takes the element-wise kernel (the 16-B path needs aligned bases): same result
    buf_e = torch.zeros(p.numel() + 1, dtype=torch.bfloat16, device=DEV)
    buf_p = torch.zeros_like(buf_e)
    buf_e[1:] = ref
    buf_p[1:] = p
    ops.ema_update(ema, p, decay, False)
    ops.ema_update(buf_e[1:], buf_p[1:], decay, False)
    torch.cuda.synchronize()
    assert torch.equal(ema, buf_e[1:])
