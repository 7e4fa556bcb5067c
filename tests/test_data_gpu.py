"""GPU parity of the bucketed data path: vpt_cover_resize_crop (libvpt_hip.so) against the CPU oracle of
the reference's transform chain (oracle/data_oracle.py: fp16 ToDtype/Normalize + ATen antialiased bicubic
via torch.nn.functional.interpolate + crop), and BucketLoader batches against per-image oracle results.

Bar (fp16 output): |diff| <= 1 fp16 ulp of the reference value (2^-10 relative, 2^-24 absolute floor),
with >= 99 % of the elements bit-identical. The f32 accumulation order differs from ATen's vectorised
CPU loops, so a last-bit flip before the single fp16 rounding is possible; nothing larger is."""

import numpy as np
import pytest
import torch

from oracle import data_oracle as DO

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def mods():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vpt import data as D
    from vpt import ops
    return D, ops


def _check(got, ref):
    got, ref = got.cpu(), ref
    assert got.shape == ref.shape
    g, r = got.float(), ref.float()
    ulp = torch.clamp(r.abs(), min=2.0 ** -14) * 2.0 ** -10
    bad = (g - r).abs() > ulp + 2.0 ** -24
    assert not bad.any(), f"{int(bad.sum())} elements beyond 1 ulp; max diff {(g - r).abs().max().item()}"
    assert (got == ref).float().mean().item() >= 0.99


@pytest.mark.parametrize("H,W,tw,th,seed", [
    (1500, 2000, 1152, 896, 0),    # 1.30x downscale, crop along the width
    (2048, 2048, 1024, 1024, 1),   # exact 2x
    (1024, 1400, 1024, 1024, 2),   # height unchanged (no vertical resample), crop along the width
    (3000, 1100, 896, 1152, 3),    # tall, 1.23x
    (4100, 5000, 1024, 1024, 4),   # ~4x downscale (17 taps)
    (700, 900, 512, 384, 5),
])
def test_cover_resize_crop_matches_oracle(mods, H, W, tw, th, seed):
    D, ops = mods
    rng = np.random.default_rng(seed)
    # smooth gradient + noise: exercises both the filter shape and the rounding path
    yy, xx = np.mgrid[0:H, 0:W]
    base = ((yy * 255 // max(H - 1, 1) + xx * 127 // max(W - 1, 1)) % 256)[..., None]
    img = np.clip(base + rng.integers(-40, 41, (H, W, 3)), 0, 255).astype(np.uint8)
    sw, sh = D.cover_size(W, H, tw, th)
    g = torch.Generator().manual_seed(seed)
    top, left = D.crop_params(sw, sh, tw, th, g)
    ref, (rsh, rsw) = DO.transform_chain(img, tw, th, top, left)
    assert (rsh, rsw) == (sh, sw)
    out = torch.empty(3, th, tw, dtype=torch.float16, device=DEV)
    D.cover_resize_crop(torch.from_numpy(img).to(DEV), tw, th, out, top, left, (sw, sh))
    torch.cuda.synchronize()
    _check(out, ref)


def test_cover_resize_crop_upscale(mods):
    D, ops = mods
    img = np.random.default_rng(7).integers(0, 256, (600, 800, 3), dtype=np.uint8)
    sw, sh = D.cover_size(800, 600, 1024, 1024, do_upscale=True)
    ref, _ = DO.transform_chain(img, 1024, 1024, 0, (sw - 1024) // 2, do_upscale=True)
    out = torch.empty(3, 1024, 1024, dtype=torch.float16, device=DEV)
    D.cover_resize_crop(torch.from_numpy(img).to(DEV), 1024, 1024, out, 0, (sw - 1024) // 2, (sw, sh))
    torch.cuda.synchronize()
    _check(out, ref)


def test_bucket_loader_batches(mods):
    """End to end: buckets, batches, crop RNG stream, and every image slot vs the oracle chain."""
    D, ops = mods
    rng = np.random.default_rng(11)
    sizes = [(int(rng.integers(1100, 1700)), int(rng.integers(1100, 1700))) for _ in range(12)]
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for (w, h) in sizes]
    loader = D.BucketLoader(imgs, sizes, [f"c{i}" for i in range(12)], batch_size=2, seed=5, device=DEV)
    gen = torch.Generator().manual_seed(5)
    order = torch.randperm(len(loader.batches), generator=gen).tolist()
    seen = 0
    for idx, batch in zip(order, loader):
        bucket, items = loader.batches[idx]
        tw, th = (int(v) for v in loader.buckets[bucket])
        assert batch["image"].shape == (2, 3, th, tw)
        assert batch["caption"] == [f"c{i}" for i in items]
        for slot, i in enumerate(items):
            w, h = sizes[i]
            sw, sh = D.cover_size(w, h, tw, th)
            top, left = D.crop_params(sw, sh, tw, th, gen)
            assert batch["crop_coords_top_left"][slot].tolist() == [top, left]
            assert batch["original_size"][slot].tolist() == [sh, sw]
            assert batch["target_size"][slot].tolist() == [th, tw]
            ref, _ = DO.transform_chain(imgs[i], tw, th, top, left)
            _check(batch["image"][slot], ref)
        seen += 1
    assert seen == len(loader)
