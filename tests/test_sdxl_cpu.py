"""CPU checks of the SDXL QLoRA oracle: the fp32 TransformerBlock + LoRALinear
restatement against the reference's own outputs (tests/golden/sdxl_block.safetensors, produced by
running src/models/sdxl/denoiser.py TransformerBlock with src/modules/peft/lora.py LoRALinear), and
the restated bitsandbytes NF4 format (parity unpinned: bitsandbytes is not installed; these are
format/round-trip properties)."""

import json
import os

import torch
from safetensors import safe_open
from safetensors.torch import load_file

from oracle import sdxl_oracle as SO

GOLD = os.path.join(os.path.dirname(__file__), "golden", "sdxl_block.safetensors")


def _fixture():
    with safe_open(GOLD, "pt") as f:
        dims = json.loads(f.metadata()["dims"])
    return load_file(GOLD), dims


def _weights(fx, d):
    w = SO.make_block_weights(d["dim"], d["heads"], d["context_dim"], d["rank"], seed=d["weight_seed"])
    for t in SO.LORA_TARGETS:
        st = {k.split("/")[-1]: v for k, v in fx.items() if k.startswith(f"nf4/{t}/")}
        w[f"{t}.linear.weight"] = SO.nf4_dequantize(st)
    return w


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_oracle_block_matches_reference_fp32():
    fx, d = _fixture()
    w = _weights(fx, d)
    x = fx["x"].clone().requires_grad_(True)
    c = fx["ctx"].clone().requires_grad_(True)
    wl = {k: (v.clone().requires_grad_(True) if "lora_" in k else v) for k, v in w.items()}
    y = SO.block_forward(x, c, wl, d["heads"], d["rank"], d["alpha"])
    (y * fx["dy"]).sum().backward()
    assert rel(y.detach(), fx["fp32/out"]) < 1e-6
    assert rel(x.grad, fx["fp32/dx"]) < 1e-6 and rel(c.grad, fx["fp32/dctx"]) < 1e-6
    n = 0
    for k, v in fx.items():
        if k.startswith("fp32/grad/"):
            assert rel(wl[k[len("fp32/grad/"):]].grad, v) < 1e-6, k
            n += 1
    assert n == 20  # lora_down + lora_up of the 10 targets
    # the reference's native bf16 run is within bf16 rounding of fp32
    assert rel(y.detach(), fx["bf16/out"]) < 2e-2


def test_nf4_fixture_states_reproduce():
    fx, d = _fixture()
    w = SO.make_block_weights(d["dim"], d["heads"], d["context_dim"], d["rank"], seed=d["weight_seed"])
    for t in SO.LORA_TARGETS:
        st = SO.nf4_quantize(w[f"{t}.linear.weight"])
        for k, v in st.items():
            assert torch.equal(v, fx[f"nf4/{t}/{k}"]), (t, k)


def test_nf4_format_properties():
    code = SO.dynamic_map()
    assert code.numel() == 256 and torch.all(code[1:] >= code[:-1]) and code.unique().numel() == 256
    assert code.min() >= -1 and code.max() == 1.0 and (code == 0).any()
    g = torch.Generator().manual_seed(3)
    w = torch.randn(96, 128, generator=g)
    st = SO.nf4_quantize(w)
    assert st["packed"].numel() == w.numel() // 2 and st["qabsmax"].numel() == w.numel() // 64
    deq = SO.nf4_dequantize(st)
    # first element of each pair in the high nibble
    first = SO.NF4[(st["packed"][0] >> 4).long()] * SO.nf4_absmax(st)[0]
    assert torch.allclose(deq.reshape(-1)[0], first)
    # round trip within half the widest NF4 gap of each block's absmax (+ the nested absmax error)
    gap = (SO.NF4[1:] - SO.NF4[:-1]).max().item()
    am = w.reshape(-1, 64).abs().amax(1, keepdim=True)
    err = (deq - w).reshape(-1, 64).abs()
    assert torch.all(err <= am * (gap / 2 + 0.02))
    assert rel(deq, w) < 0.12


def test_product_dynamic_map_equals_oracle():
    """vpt.sdxl.dynamic_map (load-time quantisation, product side) == the oracle's restatement."""
    import torch
    from oracle import sdxl_oracle as SO
    from vpt.sdxl import dynamic_map
    assert torch.equal(dynamic_map(), SO.dynamic_map())
