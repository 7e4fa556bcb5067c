"""Timestep samplers of the flow-matching step.

Restates src/modules/timestep/sampling.py (`sample_timestep`, lines 170-187, and the samplers it
dispatches to, lines 34-111 and 259-272) with an explicit torch.Generator instead of the global RNG, so
that a trainer owns its stream. Drawn with the same generator state, every sampler returns the
reference's values bit for bit (tests/test_timestep_cpu.py against tests/golden/timestep.safetensors,
produced by the reference itself). The draws are [B] f32 — no kernel: this is 8 numbers per step.
"""

from __future__ import annotations

import math

import torch

TYPES = ("shift_sigmoid", "flux_shift", "sigmoid", "uniform", "scale_shift_sigmoid")


def _lin(x: float, x1: float = 256, y1: float = 0.5, x2: float = 4096, y2: float = 1.15) -> float:
    """get_lin_function (sampling.py:9-18)."""
    m = (y2 - y1) / (x2 - x1)
    return m * x + (y1 - m * x1)


def _time_shift(mu: float, sigma: float, t: torch.Tensor) -> torch.Tensor:
    """time_shift (sampling.py:21-22)."""
    return math.exp(mu) / (math.exp(mu) + (1 / t - 1) ** sigma)


def sample_timestep(latents_shape, device=None, sampling_type: str = "sigmoid", generator: torch.Generator | None = None,
                    **kw) -> torch.Tensor:
    """t in (0, 1), shape [latents_shape[0]] f32 (sampling.py:170-187; same argument names and defaults).
    Like the reference, a sampler rejects keyword arguments it does not take, except "uniform", whose
    dispatcher call passes none on (sampling.py:170-187), so any are ignored."""
    B = int(latents_shape[0])

    def randn():
        return torch.randn(B, device=device, generator=generator)

    def take(*names):
        extra = set(kw) - set(names)
        if extra:
            raise TypeError(f"{sampling_type}: unexpected keyword arguments {sorted(extra)}")
        return kw

    if sampling_type == "shift_sigmoid":  # sampling.py:52-68
        a = take("discrete_flow_shift", "sigmoid_scale")
        shift = a.get("discrete_flow_shift", 3.1825)
        t = (randn() * a.get("sigmoid_scale", 1.0)).sigmoid()
        return (t * shift) / (1 + (shift - 1) * t)
    if sampling_type == "flux_shift":  # sampling.py:34-49
        a = take("sigmoid_scale")
        _b, _c, h, w = latents_shape
        t = (randn() * a.get("sigmoid_scale", 1.0)).sigmoid()
        return _time_shift(_lin((h // 2) * (w // 2)), 1.0, t)
    if sampling_type == "sigmoid":  # sampling.py:71-82
        a = take("sigmoid_scale")
        return (randn() * a.get("sigmoid_scale", 1.0)).sigmoid()
    if sampling_type == "uniform":  # sampling.py:85-93; the dispatcher calls uniform_rand(shape, device): kwargs dropped
        return torch.rand(B, device=device, generator=generator)
    if sampling_type == "scale_shift_sigmoid":  # sampling.py:259-272 (**kwargs swallowed there)
        std, mean = kw.get("std", 0.8), kw.get("mean", -0.8)
        return (randn() * std + mean).sigmoid()
    raise ValueError(f"Invalid sampling type: {sampling_type}")
