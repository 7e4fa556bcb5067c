"""Flat parameter / gradient storage with the reference's state-dict names.

Every parameter is a view into ONE flat bf16 buffer (and its gradient a view into ONE flat f32
buffer at the same element offset), so that
  * the GEMMs see fused operands without copies: to_q|to_k|to_v weights are adjacent ([3D, D]),
    and so are their biases, w_1|w_2 of each SwiGLU ([2F, D]) and q_norm|k_norm ([128]);
  * the optimizer and the RCCL all-reduce work on a handful of large contiguous buckets.
Names and shapes match src/models/jit/denoiser.py (JiT.__init__ 652-762) and
src/models/jit/class_encoder.py:107-121, so reference checkpoints (`denoiser.` / `class_encoder.`
prefixes, src/models/jit/pipeline.py:50-100) load unchanged.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

from .config import DenoiserConfig

ALIGN = 64  # elements; keeps every view 128-B aligned in bf16 and 256-B in f32


def _prod(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


@dataclass(frozen=True)
class ParamSpec:
    """`shape` is the reference's (logical) shape; `stored` the physical one in the flat buffer, which
    differs only for SwiGLU tensors whose hidden width F is not a multiple of 64 (e.g. JiT tiny: F =
    int(1024 * 2 / 3) = 682): they are stored zero-padded to F_pad (w_1 / w_2 rows and biases, w_3
    columns), so the GEMM operands keep 128-B aligned rows. The padding stays exactly zero through
    training (zero weights give zero activations, zero activations give zero gradients, and the
    optimizer keeps a zero parameter with zero gradient at zero)."""
    name: str
    shape: tuple
    offset: int
    stored: tuple | None = None

    @property
    def phys_shape(self) -> tuple:
        return self.stored if self.stored is not None else self.shape

    @property
    def numel(self) -> int:
        """Elements occupied in the flat buffer (physical)."""
        return _prod(self.phys_shape)


def block_param_names(i: int) -> list[str]:
    p = f"blocks.{i}."
    return [p + "attn.to_q.weight", p + "attn.to_k.weight", p + "attn.to_v.weight",
            p + "attn.to_q.bias", p + "attn.to_k.bias", p + "attn.to_v.bias",
            p + "attn.to_o.weight", p + "attn.to_o.bias",
            p + "attn.q_norm.weight", p + "attn.k_norm.weight",
            p + "norm1.weight", p + "norm2.weight",
            p + "mlp.w_1.weight", p + "mlp.w_2.weight", p + "mlp.w_1.bias", p + "mlp.w_2.bias",
            p + "mlp.w_3.weight", p + "mlp.w_3.bias"]


def param_shapes(cfg: DenoiserConfig, n_classes: int | None) -> list[tuple[str, tuple]]:
    D, F, P, C = cfg.hidden_size, cfg.mlp_hidden, cfg.patch_size, cfg.in_channels
    bd, hd = cfg.bottleneck_dim, cfg.head_dim
    out: list[tuple[str, tuple]] = [
        ("patch_embedder.proj_1.weight", (bd, C, P, P)),
        ("patch_embedder.proj_2.weight", (D, bd, 1, 1)),
        ("patch_embedder.proj_2.bias", (D,)),
        ("time_embedder.mlp.0.weight", (D, 256)), ("time_embedder.mlp.0.bias", (D,)),
        ("time_embedder.mlp.2.weight", (D, D)), ("time_embedder.mlp.2.bias", (D,)),
        ("time_position_embeds", (cfg.num_time_tokens, D)),
        ("image_size_embedder.mlp.0.weight", (D, 256)), ("image_size_embedder.mlp.0.bias", (D,)),
        ("image_size_embedder.mlp.2.weight", (D, D)), ("image_size_embedder.mlp.2.bias", (D,)),
        ("context_embedder.weight", (D, cfg.context_dim)), ("context_embedder.bias", (D,)),
    ]
    blk = {"to_q.weight": (D, D), "to_k.weight": (D, D), "to_v.weight": (D, D), "to_q.bias": (D,),
           "to_k.bias": (D,), "to_v.bias": (D,), "to_o.weight": (D, D), "to_o.bias": (D,),
           "q_norm.weight": (hd,), "k_norm.weight": (hd,), "norm1.weight": (D,), "norm2.weight": (D,),
           "w_1.weight": (F, D), "w_2.weight": (F, D), "w_1.bias": (F,), "w_2.bias": (F,),
           "w_3.weight": (D, F), "w_3.bias": (D,)}
    for i in range(cfg.depth):
        for n in block_param_names(i):
            suffix = n.split(".", 2)[2]                       # e.g. "attn.to_q.weight", "norm1.weight"
            key = suffix.split(".", 1)[1] if suffix.startswith(("attn.", "mlp.")) else suffix
            out.append((n, blk[key]))
    out += [
        ("final_layer.norm_final.weight", (D,)),
        ("final_layer.mlp.w_1.weight", (F, D)), ("final_layer.mlp.w_2.weight", (F, D)),
        ("final_layer.mlp.w_1.bias", (F,)), ("final_layer.mlp.w_2.bias", (F,)),
        ("final_layer.mlp.w_3.weight", (D, F)), ("final_layer.mlp.w_3.bias", (D,)),
        ("final_layer.linear.weight", (P * P * cfg.out_channels, D)),
        ("final_layer.linear.bias", (P * P * cfg.out_channels,)),
    ]
    if n_classes is not None:
        out.append(("class_encoder.embedding.weight", (n_classes + 1, cfg.context_dim)))
    return out


# groups of names that must be adjacent with no padding in between (fused GEMM operands)
def _contiguous_groups(cfg: DenoiserConfig) -> list[tuple[str, ...]]:
    g = []
    for i in range(cfg.depth):
        p = f"blocks.{i}."
        g += [(p + "attn.to_q.weight", p + "attn.to_k.weight", p + "attn.to_v.weight"),
              (p + "attn.to_q.bias", p + "attn.to_k.bias", p + "attn.to_v.bias"),
              (p + "attn.q_norm.weight", p + "attn.k_norm.weight"),
              (p + "mlp.w_1.weight", p + "mlp.w_2.weight"), (p + "mlp.w_1.bias", p + "mlp.w_2.bias")]
    g += [("final_layer.mlp.w_1.weight", "final_layer.mlp.w_2.weight"),
          ("final_layer.mlp.w_1.bias", "final_layer.mlp.w_2.bias")]
    return g


class ParamLayout:
    def __init__(self, cfg: DenoiserConfig, n_classes: int | None = None):
        self.cfg = cfg
        tight = set()
        for grp in _contiguous_groups(cfg):
            tight.update(grp[1:])  # members after the first follow without alignment padding
        F, Fp = cfg.mlp_hidden, cfg.mlp_hidden_padded
        specs, off = [], 0
        for name, shape in param_shapes(cfg, n_classes):
            if name not in tight:
                off = (off + ALIGN - 1) // ALIGN * ALIGN
            stored = None
            if Fp != F and ".mlp.w_" in name:
                stored = tuple(Fp if (d == F and (i == 0) == (".w_3." not in name)) else d for i, d in enumerate(shape))
            s = ParamSpec(name, shape, off, stored)
            specs.append(s)
            off += s.numel
        self.total = (off + ALIGN - 1) // ALIGN * ALIGN
        self.specs = specs
        self.by_name = {s.name: s for s in specs}

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        """The parameter in its reference shape (a strided view for column-padded w_3)."""
        s = self.by_name[name]
        v = flat[s.offset:s.offset + s.numel].view(s.phys_shape)
        if s.stored is None:
            return v
        return v[tuple(slice(0, d) for d in s.shape)]

    def phys(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        """The parameter in its stored (padded) shape, as the kernels read it."""
        s = self.by_name[name]
        return flat[s.offset:s.offset + s.numel].view(s.phys_shape)

    def span(self, flat: torch.Tensor, first: str, last: str, shape: tuple) -> torch.Tensor:
        """View spanning adjacent params first..last (a fused operand)."""
        a, b = self.by_name[first], self.by_name[last]
        assert b.offset >= a.offset
        return flat[a.offset:b.offset + b.numel].view(shape)

    def names(self) -> list[str]:
        return [s.name for s in self.specs]
