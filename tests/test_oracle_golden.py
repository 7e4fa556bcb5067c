"""CPU: pins the oracle (oracle/jit_oracle.py) against golden vectors produced by the reference
itself (tests/golden/make_golden.py) and re-expresses the reference's own known-answer tests."""

import json
import math
import os

import pytest
import torch
import torch.nn.functional as F
from safetensors import safe_open
from safetensors.torch import load_file

from oracle import jit_oracle as O
from tests.golden import golden_configs as GC

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def micro():
    return load_file(os.path.join(GOLD, "jit_micro.safetensors"))


def _run_oracle(oc, weights, fx, loss_target):
    torch.manual_seed(0)
    model = O.load_weights(O.OracleJiT(oc), weights)
    emb = weights["class_encoder.embedding.weight"].clone().requires_grad_(True)
    batch = {k: fx[k] for k in ("image", "noise", "t", "ids", "mask", "original_size", "target_size", "crop_coords")}
    loss, pred = O.train_step_loss(model, emb, batch, loss_target)
    loss.backward()
    grads = {n: p.grad for n, p in model.named_parameters()}
    grads["class_encoder.embedding.weight"] = emb.grad
    return loss.detach(), pred.detach(), grads


@pytest.fixture(scope="module")
def micro_fuse():
    return load_file(os.path.join(GOLD, "jit_micro_fuse.safetensors"))


@pytest.mark.parametrize("fuse", [False, True], ids=["strip", "fuse"])
@pytest.mark.parametrize("target", ["image", "velocity"])
def test_oracle_matches_reference_micro(micro, micro_fuse, target, fuse):
    """fuse: do_context_fuse=True (denoiser.py:1092-1113): context appended once, carried to the last block."""
    oc = GC.micro_fuse_config() if fuse else GC.micro_config()
    micro = micro_fuse if fuse else micro
    w = O.make_weights(oc, seed=1, n_classes=20)
    wsum = torch.stack([w[k].double().sum().float() for k in sorted(w)])
    assert torch.equal(wsum, micro["wsum"]), "weight generator drifted from the fixture"
    loss, pred, grads = _run_oracle(oc, w, micro, target)
    assert rel(pred, micro[f"{target}/pred"]) < 1e-5
    assert abs(loss.item() - micro[f"{target}/loss"].item()) <= 1e-5 * micro[f"{target}/loss"].item()
    for n, g in grads.items():
        gn = micro[f"{target}/gnorm/{n}"].item()
        assert abs(g.norm().item() - gn) <= 1e-4 * gn + 1e-12, n
        assert rel(g.reshape(-1)[:64], micro[f"{target}/ghead/{n}"]) < 1e-3 or gn < 1e-9, n
        if f"{target}/gfull/{n}" in micro:
            assert rel(g.reshape(-1), micro[f"{target}/gfull/{n}"]) < 1e-4, n


OBJECTIVES = {"vpred": ("velocity", "velocity", ()), "lowres_x": ("image", "image", (0.5, 0.25)),
              "lowres_v": ("image", "velocity", (0.5,))}


@pytest.mark.parametrize("case", list(OBJECTIVES))
def test_oracle_matches_reference_objectives(case):
    """jit_objectives: the reference's own train_step (class_to_image.py with model_pred="velocity";
    arb_class_to_image.py with lowres_loss passes) vs the oracle's train_step_loss on the same batch."""
    fx = load_file(os.path.join(GOLD, "jit_objectives.safetensors"))
    model_pred, loss_target, lowres = OBJECTIVES[case]
    oc = GC.micro_config()
    w = O.make_weights(oc, seed=1, n_classes=20)
    model = O.load_weights(O.OracleJiT(oc), w)
    emb = w["class_encoder.embedding.weight"].clone().requires_grad_(True)
    batch = {k: fx[f"{case}/in/{k}"] for k in ("image", "noise", "t", "ids", "mask", "original_size", "target_size",
                                               "crop_coords")}
    loss, pred = O.train_step_loss(model, emb, batch, loss_target, model_pred=model_pred, lowres_loss=lowres)
    loss.backward()
    grads = {n: p.grad for n, p in model.named_parameters()}
    grads["class_encoder.embedding.weight"] = emb.grad
    assert rel(pred.detach(), fx[f"{case}/pred"]) < 1e-5
    assert abs(loss.item() - fx[f"{case}/loss"].item()) <= 1e-5 * fx[f"{case}/loss"].item()
    for n, g in grads.items():
        gn = fx[f"{case}/gnorm/{n}"].item()
        assert abs(g.norm().item() - gn) <= 1e-4 * gn + 1e-12, n
        if f"{case}/gfull/{n}" in fx and gn > 1e-9:
            assert rel(g.reshape(-1), fx[f"{case}/gfull/{n}"]) < 1e-4, n


def test_objectives_fixture_branches_differ():
    """The velocity-prediction objective and the lowres passes change the loss (the branches are exercised)."""
    fx = load_file(os.path.join(GOLD, "jit_objectives.safetensors"))
    micro = load_file(os.path.join(GOLD, "jit_micro.safetensors"))
    assert abs(fx["vpred/loss"].item() - micro["velocity/loss"].item()) > 1e-2 * micro["velocity/loss"].item()
    assert abs(fx["lowres_x/loss"].item() - fx["lowres_v/loss"].item()) > 1e-3


def test_fuse_fixture_differs_from_strip(micro, micro_fuse):
    """The two context modes give different outputs on the same weights and batch (the branch is exercised)."""
    assert rel(micro_fuse["image/pred"], micro["image/pred"]) > 1e-3


def test_oracle_matches_reference_c1():
    fx = load_file(os.path.join(GOLD, "jit_c1.safetensors"))
    oc = GC.c1_config()
    w = O.make_weights(oc, seed=3, n_classes=1000)
    batch = GC.make_batch(oc, 4, 256, 256, 64, 1000, seed=4, padded_rows=(1, 3))
    loss, pred, grads = _run_oracle(oc, w, batch, "image")
    assert abs(loss.item() - fx["loss"].item()) <= 1e-5 * fx["loss"].item()
    assert abs(pred.double().sum().item() - fx["pred_sum"].item()) <= 1e-3 * abs(fx["pred_sq"].item()) ** 0.5
    assert rel(pred.reshape(-1)[:256], fx["pred_head"]) < 1e-5
    assert rel(pred.reshape(-1)[-256:], fx["pred_tail"]) < 1e-5
    for n, g in grads.items():
        gn = fx[f"gnorm/{n}"].item()
        assert abs(g.norm().item() - gn) <= 1e-4 * gn + 1e-12, n


# ------------------------------------------------------------------ per-op vectors
@pytest.fixture(scope="module")
def opsfx():
    path = os.path.join(GOLD, "ops.safetensors")
    with safe_open(path, "pt") as f:
        meta = f.metadata()
    return load_file(path), meta


def test_timestep_embedding_vs_reference(opsfx):
    fx, _ = opsfx
    assert torch.equal(O.timestep_embedding(fx["temb/t"]), fx["temb/out"])


def test_timestep_embedding_glide_bit_exact():
    """tests/models/test_jit.py:32-71: equals the GLIDE formula bit-exactly for t = 0..9999."""
    t = torch.arange(0, 10000)
    half = 128
    freqs = torch.exp(-math.log(10000) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
    args = t[:, None].float() * freqs[None]
    ref = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    assert torch.equal(O.timestep_embedding(t), ref)


@pytest.mark.parametrize("wh", [(256, 256), (512, 512), (1024, 1024), (960, 1088), (1088, 960), (896, 1152), (1152, 896)])
def test_rope_tables_vs_reference(opsfx, wh):
    fx, _ = opsfx
    W, H = wh
    key = f"rope/{W}x{H}"
    fc = O.rope_freqs(O.jit_b16(), H // 16, W // 16, 64)
    assert fc.shape[0] == fx[key + "/n"].item()
    assert torch.equal(torch.view_as_real(fc[:8]), fx[key + "/head"])
    assert torch.equal(torch.view_as_real(fc[-80:]), fx[key + "/tail"])
    ref_sum = fx[key + "/cos_sum"].item()  # stored as f32
    assert abs(fc.real.double().sum().item() - ref_sum) <= 1e-6 * abs(ref_sum) + 1e-3


def test_rope_apply_and_rmsnorm_vs_reference(opsfx):
    fx, _ = opsfx
    fc = torch.view_as_complex(fx["rope_apply/freqs"])
    assert torch.equal(O.apply_rope(fx["rope_apply/x"], fc), fx["rope_apply/out"])
    n = O.RMSNorm(64)
    with torch.no_grad():
        n.weight.copy_(fx["rms/w"])
    assert torch.equal(n(fx["rope_apply/x"]).detach(), fx["rms/out"])


def test_tokenizer_vs_reference(opsfx):
    fx, meta = opsfx
    caps = json.loads(meta["captions"])
    l2i = json.loads(meta["label2id"])
    ids, mask = O.class_tokenize(caps, l2i, 8)
    assert torch.equal(ids, fx["tok/ids"])
    assert torch.equal(mask, fx["tok/mask"])


@pytest.mark.parametrize("args", [(1024 ** 2, 1024, 64, 64), (64 ** 2, 64, 64, 64), (1024 ** 2, 1024, 64, 384),
                                  (256 ** 2, 256, 128, 256)])
def test_buckets_vs_reference(opsfx, args):
    fx, _ = opsfx
    ref = fx["buckets/" + "_".join(map(str, args))]
    assert torch.equal(torch.tensor(O.generate_buckets(*args)), ref)


def test_bucket_counts_known_answer():
    """tests/test_dataset.py:19-44: base 1024/step 64/min 64 -> 31 buckets; base 64 -> 1."""
    assert len(O.generate_buckets(1024 * 1024, 1024, 64, 64)) == 31
    assert len(O.generate_buckets(64 * 64, 64, 64, 64)) == 1


def test_patchify_unpatchify_roundtrip_known_answer():
    """tests/test_patch.py:17-89 idiom: exact round trip; plus conv im2col order = proj_1 weight view."""
    img = torch.randn(2, 3, 64, 96)
    p = O.patchify_conv_order(img)
    conv = torch.nn.Conv2d(3, 5, 16, 16, bias=False)
    ref = conv(img).flatten(2).transpose(1, 2)
    assert torch.allclose(p @ conv.weight.view(5, -1).t(), ref, atol=1e-5)
    q = img.view(2, 3, 4, 16, 6, 16).permute(0, 2, 4, 3, 5, 1).reshape(2, 24, 768)
    assert torch.equal(O.unpatchify(q, 64, 96), img)


def test_rope_out_of_range_bucket_raises():
    """SURVEY gotcha #8: buckets wider than 2048 px overflow rope_axes_lens=128."""
    with pytest.raises(IndexError):
        O.rope_freqs(O.jit_b16(), 2368 // 16, 448 // 16, 64)


def test_reference_bf16_error_fixture_covers_every_parameter():
    """ref_bf16_error.safetensors (the reference's own bf16-autocast step vs its fp32 step, which the GPU parity
    bar falls back to on the cancelling key-path gradients) names every gradient of each case's model."""
    import json
    from safetensors import safe_open
    from safetensors.torch import load_file
    path = os.path.join(os.path.dirname(__file__), "golden", "ref_bf16_error.safetensors")
    with safe_open(path, "pt") as f:
        names = json.loads(f.metadata()["names"])
    fx = load_file(path)
    cfgs = {"micro": (GC.micro_config(), 20), "c1": (GC.c1_config(), 1000), "jitb16-256x256-B2": (O.jit_b16(), 1000),
            "jitb16-1024x1024-B1": (O.jit_b16(), 1000)}
    for case, (oc, V) in cfgs.items():
        w = O.make_weights(oc, seed=1, n_classes=V)
        assert sorted(names[case]) == sorted(w), case
        r = fx[f"{case}/grad_rel"]
        assert r.numel() == len(w) and bool((r > 0).all()) and bool((r < 0.1).all())
        assert fx[f"{case}/loss_rel"].item() < 1e-4 and fx[f"{case}/pred_rel"].item() < 3e-2
