"""CPU checks of the sampler and checkpoint rows against the reference's own outputs
(tests/golden/sampler.safetensors, produced by running JiTModel.generate of p1atdev/vision-pt):
the oracle restatement of the Euler/CFG sampler, and the checkpoint key/shape layout."""

import json
import os

import torch
from safetensors import safe_open
from safetensors.torch import load_file

from oracle import jit_oracle as O
from tests.golden import golden_configs as GC

GOLD = os.path.join(os.path.dirname(__file__), "golden", "sampler.safetensors")


def _meta():
    with safe_open(GOLD, "pt") as f:
        return f.metadata()


def test_oracle_generate_matches_reference():
    """pipeline.py:378-488 restated: CFG 2.0, no CFG, CFG window [0.2, 0.6], velocity prediction."""
    fx = load_file(GOLD)
    cases = json.loads(_meta()["cases"])
    oc = GC.micro_config()
    w = O.make_weights(oc, seed=1, n_classes=20)
    m = O.OracleJiT(oc)
    O.load_weights(m, {k: v for k, v in w.items() if not k.startswith("class_encoder.")})
    m.eval()
    for name, kw in cases.items():
        with torch.no_grad():
            out = O.generate(m, w["class_encoder.embedding.weight"], fx["pos_ids"], fx["pos_mask"], fx["neg_ids"],
                             fx["noise"], num_inference_steps=4, cfg_scale=kw["cfg_scale"],
                             model_pred="velocity" if name.startswith("vel") else "image",
                             cfg_time_range=tuple(kw.get("cfg_time_range", (0.0, 1.0))))
        ref = fx[f"{name}/image"]
        assert ((out - ref).norm() / ref.norm()).item() < 1e-6, name


def test_tokenizer_matches_reference_prompts():
    from vpt.jit_train import ClassTokenizer
    fx = load_file(GOLD)
    prompts = json.loads(_meta()["prompts"])
    tok = ClassTokenizer({f"c{i}": i for i in range(20)})
    ids, mask = tok.tokenize(prompts, max_length=8)
    assert torch.equal(ids, fx["pos_ids"]) and torch.equal(mask, fx["pos_mask"])
    ids, mask = tok.tokenize(["", ""], max_length=8)
    assert torch.equal(ids, fx["neg_ids"]) and torch.equal(mask, fx["neg_mask"])


def test_checkpoint_layout_matches_reference_state_dict():
    """Keys and shapes written by vpt.checkpoint == JiTModel.state_dict() of the reference."""
    from vpt.config import DenoiserConfig
    from vpt.params import ParamLayout
    ref = json.loads(_meta()["state_dict"])
    oc = GC.micro_config()
    cfg = DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                         bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                         context_start_block=oc.context_start_block)
    lay = ParamLayout(cfg, n_classes=20)
    mine = {(s.name if s.name == "class_encoder.embedding.weight" else "denoiser." + s.name): list(s.shape)
            for s in lay.specs}
    assert mine == ref
