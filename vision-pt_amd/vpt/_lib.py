"""ctypes binding of the C-ABI library libvpt_hip.so (declared in include/vpt_hip.h).

The product path has no fallback: if the shared library is missing or fails to load, importing
this module raises. Every entry point returns an int status; nonzero raises RuntimeError with
`vpt_last_error_string()`.
"""

from __future__ import annotations

import ctypes as C
from pathlib import Path

from ._build import LIB, LIB_DIAG

P = C.c_void_p
L = C.c_long
I = C.c_int
F = C.c_float
U64 = C.c_ulonglong
LL = C.c_longlong

# name -> argtypes; restype is c_int unless listed in _RESTYPES.
SIGNATURES: dict[str, list] = {
    "vpt_gemm_bf16": [P, L, I, P, L, I, P, L, I, I, I, P, P, L, I, I, I, P, F, P],
    "vpt_gemm_workspace_bytes": [I, I, I, I],
    "vpt_gemm_bf16_tiled": [P, L, I, P, L, I, P, L, I, I, I, P, P, L, I, I, I, P, F, I, I, P],
    "vpt_gemm_bf16_lora": [P, L, P, L, I, P, L, P, L, I, P, L, I, I, I, P, P, L, I, I, P, I, P],
    "vpt_linear_wgrad": [P, L, P, L, P, L, P, L, I, I, I, I, P, I, I, P],
    "vpt_linear_wgrad_rr": [P, L, P, L, P, L, P, L, I, I, I, I, P, I, I, P, I, I, P, I, P],
    "vpt_linear_wgrad_workspace_bytes": [L, I, I, I],
    "vpt_gemm_swiglu_fwd": [P, L, P, L, P, P, L, P, L, I, I, I, P],
    "vpt_gemm_swiglu_bwd_workspace": [I, I, I],
    "vpt_gemm_swiglu_bwd": [P, L, P, L, P, L, P, L, I, I, I, P, P],
    "vpt_attn_fwd": [P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, P, L, I, I, I, I, I, F, P],
    "vpt_attn_bwd": [P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, P, L, L, P, L,
                     P, L, L, L, P, L, L, L, P, L, L, L, I, I, I, I, I, F, P],
    "vpt_attn_bwd_q": [P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, P, L, L, P, L,
                       P, L, L, L, P, L, L, L, P, L, L, L, I, I, I, I, I, F, P, P],
    "vpt_attn_bwd_queue_bytes": [],
    "vpt_attn_bwd_qknorm": [P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, P, L, L, P, L,
                            P, P, L, L, L, P, P, P, P, F, P, P, L, L, L, P, P, L, P, L, L, L, I, I, I, I, I, F, P],
    "vpt_attn_bwd_dw_rows": [I, I, I],
    "vpt_attn_fwd_qknorm": [P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, L, P, L, L, P, L, P, P, I, I, I, I, I, F, P],
    "vpt_linear_qknorm_rope": [P, L, P, L, P, P, L, P, L, I, I, I, P, P, P, P, I, F, F, P],
    "vpt_attn_q_scale": [F],
    "vpt_rmsnorm_fwd": [P, L, P, P, L, P, I, I, F, P],
    "vpt_rmsnorm_bwd_blocks": [I],
    "vpt_rmsnorm_bwd": [P, L, P, L, P, P, P, L, P, L, P, I, I, P],
    "vpt_qknorm_rope_blocks": [I],
    "vpt_qknorm_rope_fwd": [P, L, P, P, P, P, P, L, I, I, I, F, F, P],
    "vpt_qknorm_rope_bwd": [P, L, P, L, P, P, P, P, P, L, P, I, I, I, F, P],
    "vpt_qknorm_rope_bwd_rows": [P, L, P, L, P, P, P, P, P, L, P, I, I, I, I, F, P],
    "vpt_reduce_rows": [P, I, I, P, I, P],
    "vpt_patchify": [P, I, P, P, F, U64, I, I, I, P, P],
    "vpt_unpatchify": [P, I, I, I, P, I, P],
    "vpt_loss_blocks": [],
    "vpt_gauss_noise": [L, U64, F, P, P],
    "vpt_area_lowres": [P, P, P, F, U64, I, I, I, I, P, P, P, P],
    "vpt_euler_cfg_step": [P, P, I, I, I, I, F, I, F, F, P],
    "vpt_flow_loss": [P, P, P, P, F, U64, I, F, I, I, I, P, P, P, P],
    "vpt_timestep_embed": [P, I, P, P],
    "vpt_assemble_tokens": [P, P, P, P, P, I, I, I, I, I, P, P],
    "vpt_disassemble_tokens": [P, I, I, I, I, P, P, P, P, P],
    "vpt_ctx_rows": [P, I, I, I, I, P, P, I, I, P],
    "vpt_swiglu_fwd": [P, L, I, P, P],
    "vpt_swiglu_bwd": [P, P, L, I, P, P],
    "vpt_colsum_blocks": [L],
    "vpt_bias_grad": [P, L, L, I, P, P, I, P],
    "vpt_embed_gather": [P, P, L, I, P, P],
    "vpt_embed_scatter_add": [P, P, L, I, LL, P, P],
    "vpt_embed_grad_set": [P, P, L, I, LL, L, I, P, P],
    "vpt_step_inputs": [P, I, F, P, P, P, P, P, P, I, I, I, P, P],
    "vpt_cast_f32_bf16": [P, L, P, P],
    "vpt_radam_sf_step": [P, P, I, P, P, L, F, F, F, F, F, F, F, F, I, P, F, P],
    "vpt_grad_norm_blocks": [],
    "vpt_grad_sumsq": [P, I, L, F, P, P],
    "vpt_clip_coef": [P, I, F, P, P, P],
    "vpt_sf_lerp": [P, P, L, F, P],
    "vpt_sf_init": [P, P, P, L, P],
    "vpt_copy_rows": [P, L, I, I, I, P, L, I, I, I, P],
    "vpt_silu": [P, P, P, L, I, P],
    "vpt_layernorm_fwd": [P, L, P, P, P, L, P, P, I, I, F, P],
    "vpt_layernorm_lora_fwd": [P, L, P, P, P, L, P, P, I, I, F, P, L, I, P, L, F, P],
    "vpt_layernorm_bwd_blocks": [I],
    "vpt_layernorm_bwd": [P, L, P, L, P, P, P, P, L, P, L, P, P, I, I, P],
    "vpt_layernorm_bwd_lora": [P, L, P, L, P, P, P, P, L, P, L, I, I, P, P, L, F, P],
    "vpt_geglu_fwd": [P, L, I, L, P, P],
    "vpt_geglu_bwd": [P, P, L, I, L, P, L, P],
    "vpt_geglu_bwd_lora": [P, P, L, I, I, P, L, P, P, L, F, P, P, P],
    "vpt_geglu_lora_partials_bytes": [I, I],
    "vpt_geglu_fwd_lora": [P, L, I, I, P, L, P, P, L, F, P, P, P],
    "vpt_nf4_dequant": [P, P, P, P, P, L, P, P],
    "vpt_nf4_dequant_batch": [P, I, P],
    "vpt_scale_bf16_2d": [P, L, L, I, F, P, L, P],
    "vpt_gemm_bf16_lora_grouped": [P, L, P, L, P, L, P, I, I, P, L, I, I, I, P, P, L, I, P, I, P],
    "vpt_gemm_bf16_lora_scaled": [P, L, P, L, I, P, L, P, L, I, P, L, I, I, I, P, P, L, I, F, I, P],
    "vpt_gemm_bf16_lora_grouped_scaled": [P, L, P, L, P, L, P, I, I, P, L, I, I, I, P, P, L, I, F, I, P],
    "vpt_gemm_bf16_lora_stacked": [P, L, P, L, P, L, P, I, I, P, L, I, I, I, I, P, I, P],
    "vpt_groupnorm_fwd": [P, P, P, P, P, P, I, I, I, L, F, P],
    "vpt_groupnorm_bwd": [P, P, P, P, P, P, P, I, I, I, L, P],
    "vpt_transpose_add": [P, P, P, I, I, I, P],
    "vpt_lora_proj": [P, L, P, I, P, L, I, I, I, F, P],
    "vpt_lora_wgrad_workspace": [I, I],
    "vpt_lora_wgrad2": [P, L, P, L, P, I, P, L, P, L, P, I, I, I, F, P, P, P],
    "vpt_lora_wgrad_splits": [I, I],
    "vpt_lora_wgrad2_partial": [P, L, P, L, I, P, L, P, L, I, I, P, P, P],
    "vpt_lora_wgrad_reduce_batch": [P, I, F, I, P],
    "vpt_lora_wgrad_partial_batch": [P, I, P],
    "vpt_lora_proj_grouped": [P, L, L, P, I, L, P, L, I, I, I, I, F, P],
    "vpt_ema_update": [P, P, L, F, F, I, P],
    "vpt_gemm_nf4": [P, L, P, P, P, P, P, L, I, P, L, P, L, I, P, L, I, I, I, P, P, L, I, F, P],
    "vpt_nf4_quantize": [P, L, P, P, P, P, P, P, P],
    "vpt_add_bf16": [P, P, L, P, P],
    "vpt_flow_noise": [P, P, L, I, F, I, U64, P, P, P, P],
    "vpt_velocity_loss_blocks": [],
    "vpt_velocity_loss": [P, P, P, L, P, P, P, P],
    "vpt_sinusoid_embed": [P, I, I, P, P],
    "vpt_space_to_depth": [P, P, I, I, I, I, I, I, P],
    "vpt_scale_bf16": [P, L, F, P, P],
    "vpt_cover_resize_crop_workspace": [I, I, I, I, I, I, I],
    "vpt_cover_resize_crop": [P, I, I, I, I, I, I, I, I, P, P, P],
    "vpt_last_error_string": [],
    "vpt_abi_version": [],
    "vpt_build_info": [],
}
# Diagnostic-only entry points (include/vpt_hip_diag.h): exported by libvpt_hip_diag.so, loaded only
# explicitly by tools/ (use_diag()), never by the product path.
DIAG_SIGNATURES: dict[str, list] = {
    "vpt_gemm_set_geometry": [I],
    "vpt_gemm_set_stagger": [I],
    "vpt_gemm_set_debug": [P],
    "vpt_gemm_set_ring_grid": [I],
    "vpt_attn_set_rescale_threshold": [F],
    "vpt_attn_set_variant": [I],
    "vpt_attn_fused_workspace_bytes": [I, I, I],
    "vpt_attn_set_fused_workspace": [P],
    "vpt_attn_set_rows64": [I],
    "vpt_attn_set_bwd_stages": [I],
    "vpt_attn_set_xcd_order": [I],
    "vpt_attn_set_fwd_order": [I],
    "vpt_attn_set_bwd_prefetch": [I],
    "vpt_attn_set_bwd_partner": [I],
    "vpt_attn_set_fwd_lsum": [I],
    "vpt_attn_set_bwd_mfma16": [I],
    "vpt_attn_set_fwd_mfma16": [I],
    "vpt_gemm_set_swb_one_group": [I],
    "vpt_gemm_set_swb_ablation": [I],
    "vpt_gemm_set_r2": [I],
    "vpt_gemm_set_nf4_ablation": [I],
    "vpt_diag_occupy": [I, L, I, P, P],
}
_RESTYPES = {
    "vpt_lora_wgrad_workspace": C.c_long,
    "vpt_geglu_lora_partials_bytes": C.c_long,
    "vpt_gemm_workspace_bytes": C.c_long,
    "vpt_linear_wgrad_workspace_bytes": C.c_long,
    "vpt_attn_fused_workspace_bytes": C.c_long,
    "vpt_cover_resize_crop_workspace": C.c_long,
    "vpt_gemm_swiglu_bwd_workspace": C.c_long,
    "vpt_attn_q_scale": C.c_float,
    "vpt_last_error_string": C.c_char_p,
    "vpt_build_info": C.c_char_p,
}
# Entry points that return a value (size / count / string) rather than a status code.
_VALUE_FNS = {"vpt_attn_bwd_queue_bytes", "vpt_grad_norm_blocks", "vpt_velocity_loss_blocks", "vpt_lora_wgrad_workspace", "vpt_geglu_lora_partials_bytes", "vpt_lora_wgrad_splits", "vpt_gemm_workspace_bytes", "vpt_linear_wgrad_workspace_bytes", "vpt_attn_fused_workspace_bytes", "vpt_cover_resize_crop_workspace", "vpt_gemm_swiglu_bwd_workspace", "vpt_rmsnorm_bwd_blocks", "vpt_layernorm_bwd_blocks", "vpt_qknorm_rope_blocks", "vpt_loss_blocks",
              "vpt_colsum_blocks", "vpt_attn_q_scale", "vpt_attn_bwd_dw_rows", "vpt_last_error_string", "vpt_abi_version", "vpt_build_info"}


def _load(path: Path, diag: bool = False) -> C.CDLL:
    if not path.exists():
        raise ImportError(
            f"{path} not found: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = C.CDLL(str(path))
    sigs = {**SIGNATURES, **DIAG_SIGNATURES} if diag else SIGNATURES
    for name, args in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, C.c_int)
    return lib


ABI_VERSION = 5  # the signatures in SIGNATURES / include/vpt_hip.h


def load_library(path: Path | str, diag: bool = False) -> C.CDLL:
    """Loads one build of the C ABI and checks its ABI version (does not route calls through it)."""
    path = Path(path)
    lib_ = _load(path, diag)
    if lib_.vpt_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: ABI {lib_.vpt_abi_version()} != {ABI_VERSION} expected by these bindings; rebuild it")
    return lib_


# The product library. No environment read and no fallback: tools/ that need the diagnostic twin (or another build of
# the same sources, for a compile-flag A/B) switch to it explicitly with use_library() / use_diag().
DIAG = False
LIB_PATH = LIB
lib = load_library(LIB)


def use_library(lib_or_path, diag: bool = False) -> C.CDLL:
    """tools/ only: routes every later call() through another build (a loaded CDLL or a path)."""
    global lib, LIB_PATH, DIAG
    if isinstance(lib_or_path, C.CDLL):
        lib = lib_or_path
        LIB_PATH = Path(lib_or_path._name)
    else:
        lib = load_library(lib_or_path, diag)
        LIB_PATH = Path(lib_or_path)
    DIAG = diag
    return lib


def use_diag() -> C.CDLL:
    """tools/ only: the -DVPT_DIAG twin libvpt_hip_diag.so (process-wide A/B switches, timing ablations)."""
    return use_library(LIB_DIAG, diag=True)


def call(name: str, *args):
    """Calls a status-returning entry point; raises RuntimeError on a nonzero status."""
    rc = getattr(lib, name)(*args)
    if name in _VALUE_FNS:
        return rc
    if rc != 0:
        msg = lib.vpt_last_error_string().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")
    return rc
