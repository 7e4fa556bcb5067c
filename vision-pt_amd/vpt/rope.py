"""RoPE frequency tables per bucket, built once on the host and cached on the device.

Restates RopeEmbedder (src/models/jit/denoiser.py:114-287): per axis (dims 16/24/24 -> 8/12/12
complex frequencies) freq_j = theta^(-2j/d) in f64, angle = pos * freq in f64 cast to f32,
polar(1, angle) in f32. Image axes are zero-centred: y in [h_p//2 - h_p, h_p//2); context, time
and image-size tokens use (global index, i, i). Token order patches | size(6) | time(T) | context
(denoiser.py:1032-1051). The reference rebuilds this on the CPU and copies [B,N,32] complex64 to
the GPU every forward; here it is one [rows,32] cos table + one sin table per bucket.
"""

from __future__ import annotations

import torch

from .config import DenoiserConfig


def _axis_angles(dim: int, lo: int, hi: int, theta: float) -> torch.Tensor:
    freqs = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    pos = torch.arange(lo, hi, dtype=torch.float64)
    return torch.outer(pos, freqs).float()


def rope_angles(cfg: DenoiserConfig, h_p: int, w_p: int, n_ctx: int) -> torch.Tensor:
    """f32 angles [N, head_dim/2] in token order."""
    tabs, offs = [], []
    for dim, ln, zc in zip(cfg.rope_axes_dims, cfg.rope_axes_lens, cfg.rope_zero_centered):
        lo, hi = ((ln // 2) - ln, ln // 2) if zc else (0, ln)
        tabs.append(_axis_angles(dim, lo, hi, cfg.rope_theta))
        offs.append(ln // 2 if zc else 0)

    def lookup(ids: torch.Tensor) -> torch.Tensor:
        cols = []
        for a in range(len(tabs)):
            idx = ids[:, a] + offs[a]
            if int(idx.min()) < 0 or int(idx.max()) >= tabs[a].shape[0]:
                raise ValueError(
                    f"RoPE axis {a} position out of range for a {h_p}x{w_p}-patch bucket "
                    f"(rope_axes_lens={cfg.rope_axes_lens}); the reference fails in torch.gather here")
            cols.append(tabs[a][idx])
        return torch.cat(cols, -1)

    ys = torch.arange(h_p // 2 - h_p, h_p // 2).view(-1, 1).expand(h_p, w_p)
    xs = torch.arange(w_p // 2 - w_p, w_p // 2).view(1, -1).expand(h_p, w_p)
    img = torch.stack([torch.full_like(ys, 3), ys, xs], -1).reshape(-1, 3)

    def seq(n: int, g: int) -> torch.Tensor:
        a = torch.arange(n)
        return torch.stack([torch.full_like(a, g), a, a], -1)

    parts = [img, seq(6, 2), seq(cfg.num_time_tokens, 1)]
    if n_ctx:
        parts.append(seq(n_ctx, 0))
    return torch.cat([lookup(p) for p in parts], 0)


class RopeCache:
    """(h_p, w_p, n_ctx) -> (cos, sin) device tables [rows, 32] f32."""

    def __init__(self, cfg: DenoiserConfig, device):
        self.cfg = cfg
        self.device = device
        self._cache: dict[tuple[int, int, int], tuple[torch.Tensor, torch.Tensor]] = {}

    def get(self, h_p: int, w_p: int, n_ctx: int):
        key = (h_p, w_p, n_ctx)
        if key not in self._cache:
            ang = rope_angles(self.cfg, h_p, w_p, n_ctx)
            c = torch.polar(torch.ones_like(ang), ang)  # f32 cos/sin exactly as torch.polar computes them
            self._cache[key] = (c.real.contiguous().to(self.device), c.imag.contiguous().to(self.device))
        return self._cache[key]
