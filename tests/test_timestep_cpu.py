"""a1: vpt.timestep.sample_timestep vs the reference's own draws (tests/golden/timestep.safetensors, made by
tests/golden/make_golden.py timestep from src/modules/timestep/sampling.py). Same RNG state -> bit-exact."""
import json
import os
import sys

import pytest
import torch
from safetensors import safe_open

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

from vpt.timestep import sample_timestep  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "timestep.safetensors")


def _cases():
    with safe_open(GOLD, "pt") as f:
        cases = json.loads(f.metadata()["cases"])
        return [(k, f.get_tensor(k), cases) for k in f.keys()]


@pytest.mark.parametrize("key,ref,cases", _cases(), ids=lambda v: v if isinstance(v, str) else "")
def test_sampler_matches_reference(key, ref, cases):
    name, shape, seed = key.split("/")
    typ = name.split("_m0")[0].split("_s2")[0]
    g = torch.Generator().manual_seed(int(seed))
    t = sample_timestep(tuple(int(s) for s in shape.split("x")), "cpu", typ, generator=g, **cases[name])
    assert t.dtype == torch.float32 and t.shape == ref.shape
    assert torch.equal(t, ref), (t - ref).abs().max()


def test_sampler_rejects_foreign_kwargs():
    # the reference's sigmoid_randn has no mean/std parameters (sampling.py:71-82): TypeError there too
    with pytest.raises(TypeError):
        sample_timestep((4, 3, 8, 8), "cpu", "sigmoid", mean=0.0)
    with pytest.raises(ValueError):
        sample_timestep((4, 3, 8, 8), "cpu", "bogus")


def test_uniform_ignores_kwargs_like_the_dispatcher():
    # sampling.py:183-184 calls uniform_rand(latents_shape, device) without **kwargs
    from vpt.timestep import sample_timestep
    a = sample_timestep((5, 3, 8, 8), "cpu", "uniform", generator=torch.Generator().manual_seed(1), sigmoid_scale=2.0)
    b = sample_timestep((5, 3, 8, 8), "cpu", "uniform", generator=torch.Generator().manual_seed(1))
    assert torch.equal(a, b) and a.shape == (5,)


def test_scale_shift_sigmoid_distribution():
    # JiT's sampler (config.yml timestep_sampling): logit-normal with mean -0.8, std 0.8
    t = sample_timestep((200000, 3, 8, 8), "cpu", "scale_shift_sigmoid", generator=torch.Generator().manual_seed(1))
    logit = torch.log(t / (1 - t))
    assert abs(logit.mean().item() + 0.8) < 0.01 and abs(logit.std().item() - 0.8) < 0.01
