"""Config surface mirrored from the reference (same field names / defaults, so the reference's
YAML `model.denoiser:` dicts validate unchanged).

  DenoiserConfig      <- src/models/jit/config.py:16-46
  JiT_B_16_Config     <- src/models/jit/config.py:49-65
  JiTTrainingConfig   <- train/jit/arb_class_to_image.py:26-44 (JiTConfigForTraining, every field, including the
                         inherited JiTConfig ones of src/models/jit/config.py:95-102); unknown keys are refused
                         (extra="forbid") instead of silently dropped, and the reference's known values this path
                         does not build raise NotImplementedError as the reference's own treat_loss does
"""

from __future__ import annotations

from typing import Literal

from pydantic import BaseModel, ConfigDict, field_validator, model_validator

NormType = Literal["layer", "rms", "dyt", "derf"]
PositionalEncoding = Literal["rope", "pope", "n-pope"]


class DenoiserConfig(BaseModel):
    patch_size: int = 16
    in_channels: int = 3
    out_channels: int = 3
    hidden_size: int = 1024
    depth: int = 24
    num_heads: int = 16
    mlp_ratio: float = 4.0
    attn_dropout: float = 0.0
    proj_dropout: float = 0.0

    bottleneck_dim: int = 128
    use_output_bottleneck: bool = False
    use_pixel_shuffle: bool = False

    norm_type: NormType = "rms"

    num_time_tokens: int = 4
    timestep_scale: float = 1.0

    positional_encoding: PositionalEncoding = "rope"
    rope_theta: float = 256.0
    rope_axes_dims: list[int] = [16, 24, 24]
    rope_axes_lens: list[int] = [256, 128, 128]
    rope_zero_centered: list[bool] = [False, True, True]
    rope_do_normalize: list[bool] = [False, True, True]
    rope_normalize_by: float = 64.0

    context_dim: int = 768
    context_start_block: int = 0
    do_context_fuse: bool = False

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def mlp_hidden(self) -> int:
        # SwiGLU(dim, hidden_dim=int(D*mlp_ratio)) uses int(hidden_dim * 2 / 3) (denoiser.py:490, 641-646)
        return int(int(self.hidden_size * self.mlp_ratio) * 2 / 3)

    @property
    def mlp_hidden_padded(self) -> int:
        """SwiGLU hidden width as stored and computed (zero-padded to a multiple of 64; vpt.params)."""
        return (self.mlp_hidden + 63) // 64 * 64


class JiT_B_16_Config(DenoiserConfig):
    patch_size: int = 16
    depth: int = 12
    hidden_size: int = 768
    num_heads: int = 12
    bottleneck_dim: int = 128
    context_dim: int = 768
    context_start_block: int = 4
    rope_axes_dims: list[int] = [16, 24, 24]
    rope_axes_lens: list[int] = [256, 128, 128]


class JiTTrainingConfig(BaseModel):
    """The `model:` section of a JiT training YAML (configs/jit/x-loss/config.yml). Objectives: model_pred "image"
    with loss_target "image" | "velocity" (arb_class_to_image.py:108-147), model_pred "velocity" with loss_target
    "velocity" (class_to_image.py:146-156: target clean - noise, no timestep clamp); lowres_loss adds one pass per
    scale on area-resized inputs (arb_class_to_image.py:228-272)."""

    model_config = ConfigDict(extra="forbid")

    # JiTConfig (src/models/jit/config.py:95-102)
    dtype: str = "float32"
    context_encoder: dict | None = None
    denoiser: DenoiserConfig = JiT_B_16_Config()
    model_pred: Literal["image", "velocity", "noise"] = "image"
    # JiTConfigForTraining (train/jit/arb_class_to_image.py:26-40)
    checkpoint_path: str | None = None
    max_token_length: int = 64
    noise_scale: float = 1.0
    timestep_eps: float = 0.05
    loss_target: Literal["velocity", "image"] = "velocity"
    timestep_sampling: str = "scale_shift_sigmoid"
    train_class_encoder: bool = True
    drop_context_rate: float = 0.1
    lowres_loss: list[float] = []

    @field_validator("context_encoder")
    @classmethod
    def _class_context(cls, v):
        if v is not None and v.get("type", "class") != "class":
            raise NotImplementedError("HIP JiT: only the class context encoder (text encoders are out of scope)")
        return v

    @model_validator(mode="after")
    def _objective(self):
        if self.model_pred == "noise":  # class_to_image.py:161-162
            raise NotImplementedError("Noise prediction is not implemented yet.")
        if self.model_pred == "velocity" and self.loss_target != "velocity":  # class_to_image.py:157-160
            raise NotImplementedError("Velocity prediction with image loss is not implemented yet.")
        for s in self.lowres_loss:
            if s > 0.0:
                lowres_factor(s)
        return self

    @property
    def loss_kind(self) -> int:
        """vpt_flow_loss target: 0 image loss, 1 velocity loss of an image prediction, 2 velocity prediction."""
        if self.model_pred == "velocity":
            return 2
        return 0 if self.loss_target == "image" else 1


def lowres_factor(scale: float) -> int:
    """The integer area-pooling factor k of a lowres_loss scale (F.interpolate(scale_factor=scale, mode="area") with
    scale = 1/k): the HIP path builds even k (2, 4, 6, ...: whole pixel pairs of the noise generator)."""
    k = round(1.0 / scale)
    if k < 2 or k % 2 or abs(k * scale - 1.0) > 1e-9:
        raise NotImplementedError(f"HIP JiT: lowres_loss scale {scale} must be 1/k for an even integer k")
    return k


def check_supported(cfg: DenoiserConfig) -> None:
    """The HIP path implements the JiT-B family path of the reference; reject the variants it
    does not (they raise instead of silently computing something else)."""
    if cfg.positional_encoding != "rope":
        raise NotImplementedError("HIP JiT: only positional_encoding='rope' (PoPE variants are out of scope)")
    if cfg.norm_type != "rms":
        raise NotImplementedError("HIP JiT: only norm_type='rms'")
    if cfg.use_output_bottleneck or cfg.use_pixel_shuffle:
        raise NotImplementedError("HIP JiT: output bottleneck / pixel shuffle heads are out of scope")
    if cfg.head_dim != 64 or sum(cfg.rope_axes_dims) != 64:
        raise NotImplementedError("HIP JiT: head_dim must be 64 (rope_axes_dims summing to 64)")
    if cfg.patch_size != 16 or cfg.in_channels != 3 or cfg.out_channels != 3:
        raise NotImplementedError("HIP JiT: patch 16, 3 channels")
    if cfg.hidden_size % 64 or cfg.context_dim % 8 or cfg.bottleneck_dim % 8:
        raise NotImplementedError("HIP JiT: hidden_size % 64, context_dim % 8, bottleneck_dim % 8")
    if cfg.attn_dropout != 0.0 or cfg.proj_dropout != 0.0:
        raise NotImplementedError("HIP JiT: dropout must be 0 (reference default)")
    if len(cfg.rope_axes_dims) != 3:
        raise NotImplementedError("HIP JiT: 3 rope axes")
