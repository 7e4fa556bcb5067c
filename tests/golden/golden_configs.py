"""Configs and synthetic batches shared by the golden generator and the tests (no reference import)."""

import torch

from oracle.jit_oracle import OracleConfig


def micro_config() -> OracleConfig:
    return OracleConfig(hidden_size=192, depth=3, num_heads=3, bottleneck_dim=32, context_dim=64,
                        context_start_block=1)


def micro_fuse_config() -> OracleConfig:
    """micro_config with do_context_fuse=True (denoiser.py:1092-1113, config.py:46)."""
    return OracleConfig(hidden_size=192, depth=3, num_heads=3, bottleneck_dim=32, context_dim=64,
                        context_start_block=1, do_context_fuse=True)


def c1_config() -> OracleConfig:
    """BASELINE config 1: JiT tiny (2 layers, d=256), context in both blocks."""
    return OracleConfig(hidden_size=256, depth=2, num_heads=4, bottleneck_dim=128, context_dim=256,
                        context_start_block=0)


def make_batch(oc: OracleConfig, B, H, W, n_ctx, n_classes, seed, padded_rows=(1,)):
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).half()
    noise = torch.randn(B, 3, H, W, generator=g).half()
    t = (torch.randn(B, generator=g) * 0.8 - 0.8).sigmoid()
    ids = torch.randint(0, n_classes, (B, n_ctx), generator=g)
    mask = torch.ones(B, n_ctx, dtype=torch.long)
    for r in padded_rows:
        if r < B:
            keep = max(1, n_ctx // 2 - r)
            ids[r, keep:] = n_classes  # pad id
            mask[r, keep:] = 0
    sizes = torch.tensor([[H, W]]).repeat(B, 1)
    return dict(image=x, noise=noise, t=t, ids=ids, mask=mask, original_size=sizes, target_size=sizes.clone(),
                crop_coords=torch.zeros(B, 2, dtype=torch.long))
