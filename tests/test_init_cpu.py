"""a27: JiTEngine.init_weights vs the reference's JiT.initialize_weights + ClassEncoder.initialize_weights
(tests/golden/init.safetensors, made from the reference by tests/golden/make_golden.py init): every parameter
is drawn from the same distribution (ones / zeros / N(0, 0.02)), key for key. Host only (no kernels)."""
import json
import math
import os
import sys

import torch
from safetensors import safe_open

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

from tests.golden import golden_configs as GC  # noqa: E402
from vpt.config import DenoiserConfig  # noqa: E402
from vpt.engine import JiTEngine  # noqa: E402


def test_init_matches_reference_distribution():
    with safe_open(os.path.join(ROOT, "tests", "golden", "init.safetensors"), "pt") as f:
        names = json.loads(f.metadata()["names"])
        stats = f.get_tensor("stats")
    oc = GC.micro_config()
    cfg = DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                         bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                         context_start_block=oc.context_start_block)
    eng = JiTEngine(cfg, device="cpu", n_classes=20)
    eng.init_weights(seed=5)
    assert sorted(eng.p) == names  # identical state-dict keys, class encoder included
    for n, (kind, mean, std, numel) in zip(names, stats.tolist()):
        t = eng.p[n].double()
        assert t.numel() == int(numel), n
        if kind == 1:
            assert bool((t == 1).all()), n
        elif kind == 2:
            assert bool((t == 0).all()), n
        else:
            # N(0, 0.02) (bf16-rounded on our side): sampling error of the std ~ 0.02 / sqrt(2 numel)
            tol = 6 * 0.02 / math.sqrt(2 * numel) + 2e-4
            assert abs(std - 0.02) < tol, (n, std)
            assert abs(t.std().item() - 0.02) < tol, (n, t.std().item())
            assert abs(t.mean().item()) < 6 * 0.02 / math.sqrt(numel) + 1e-5, n


def test_init_is_seeded():
    oc = GC.micro_config()
    cfg = DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                         bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                         context_start_block=oc.context_start_block)
    a, b = JiTEngine(cfg, device="cpu", n_classes=20), JiTEngine(cfg, device="cpu", n_classes=20)
    a.init_weights(seed=3)
    b.init_weights(seed=3)
    assert torch.equal(a.params, b.params)  # every rank starts from the same weights (DDP broadcast stand-in)
