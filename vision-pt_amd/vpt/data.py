"""Aspect-ratio-bucketed training batches, device-side.

Host bookkeeping mirrors the reference exactly (bucket enumeration, nearest-bucket assignment, the
per-bucket pre-batched slicing with its modulo semantics, the ConcatDataset + batch_size=1 loader with
concatenating collate); the per-image transform chain runs on the GPU (`vpt_cover_resize_crop`):

  reference (CPU, per image)                                  here
  src/dataset/aspect_ratio_bucket.py:20-60  generate_buckets   generate_buckets
  src/dataset/aspect_ratio_bucket.py:89-155 find_nearest       AspectRatioBucketManager.find_nearest
  src/dataset/bucket.py:45-121  Bucket / BucketDataset          BucketBatches (index -> item indices)
  src/dataset/text_to_image.py:445-505  generate_buckets        assign_buckets
  src/dataset/text_to_image.py:145-158,199-213 + transform.py:11-55
      PILToTensor, ToDtype(fp16), Normalize, ObjectCoverResize (bicubic AA), RandomCrop
                                                                cover_size + crop_params + ops.cover_resize_crop
  src/dataloader.py:33-49,68-87  DataLoader(bs=1) + concatnate_collate_fn
                                                                BucketLoader (one bucket batch per step)

Decoding stays on the host (PIL); decoded uint8 HWC arrays are uploaded and transformed in HBM, and each
image lands directly in its [B,3,h,w] fp16 batch slot.
"""

from __future__ import annotations

import math
from typing import Callable, Sequence

import numpy as np
import torch

from . import ops


# ----------------------------------------------------------------------------- buckets
def generate_buckets(target_area: int = 1024 * 1024, start_size: int = 1024, step: int = 64,
                     min_size: int = 64) -> np.ndarray:
    """(width, height) pairs of ~target_area with both sides multiples of `step`
    (src/dataset/aspect_ratio_bucket.py:20-60): widths descend from start_size; the height is the area
    quotient rounded to a multiple of step; stop once it falls below min_size; non-square pairs are added
    in both orientations."""
    out = []
    w = start_size
    while w >= min_size:
        h = round(target_area / w / step) * step
        if h < min_size:
            break
        out.append(np.array([w, h]))
        if w != h:
            out.append(np.array([h, w]))
        w -= step
    return np.stack(out)


class AspectRatioBucketManager:
    """src/dataset/aspect_ratio_bucket.py:89-155."""

    def __init__(self, buckets: np.ndarray):
        self.buckets = buckets
        self.aspect_ratios = np.log2(buckets[:, 0] / buckets[:, 1])
        self.resolutions = buckets[:, 0] * buckets[:, 1]
        self.sorted_indices = np.argsort(-self.resolutions)

    def __len__(self) -> int:
        return self.buckets.shape[0]

    def find_nearest(self, width: int, height: int) -> int:
        """Bucket no larger than the image on either side with the closest log2 aspect ratio; ties keep
        the first in descending-resolution order. Raises when none fits (reference: AssertionError)."""
        ar = math.log2(width / height)
        best, best_diff = None, float("inf")
        for idx in self.sorted_indices:
            bw, bh = self.buckets[idx]
            if bw > width or bh > height:
                continue
            diff = abs(ar - self.aspect_ratios[idx])
            if diff < best_diff:
                best, best_diff = idx, diff
        if best is None:
            raise AssertionError(f"No bucket found for image size {width}x{height}")
        return int(best)


def assign_buckets(sizes: Sequence[tuple[int, int]], buckets: np.ndarray) -> dict[int, list[int]]:
    """Item index lists per bucket index, in item order (text_to_image.py:461-476); items too small for
    every bucket are skipped, as the reference does (with a warning there)."""
    mgr = AspectRatioBucketManager(buckets)
    out: dict[int, list[int]] = {}
    for i, (w, h) in enumerate(sizes):
        try:
            b = mgr.find_nearest(w, h)
        except AssertionError:
            continue
        out.setdefault(b, []).append(i)
    return out


class BucketBatches:
    """The reference's ConcatDataset([BucketDataset(bucket) ...]) index space (bucket.py:45-121,
    text_to_image.py:484-512): bucket k contributes ceil(num_items * num_repeats / batch_size) entries;
    entry idx of bucket k is items[(real*bs + j) % num_items] for j < bs, real = idx % num_items."""

    def __init__(self, subsets: dict[int, list[int]], batch_size: int, num_repeats: int = 1):
        self.buckets = [(b, items) for b, items in subsets.items() if len(items) > 0]
        self.batch_size = batch_size
        self.lengths = [math.ceil(len(items) * num_repeats / batch_size) for _, items in self.buckets]
        self.offsets = np.cumsum([0] + self.lengths)

    def __len__(self) -> int:
        return int(self.offsets[-1])

    def __getitem__(self, idx: int) -> tuple[int, list[int]]:
        if idx < 0 or idx >= len(self):
            raise IndexError(idx)
        k = int(np.searchsorted(self.offsets, idx, side="right") - 1)
        local = idx - int(self.offsets[k])
        bucket, items = self.buckets[k]
        n = len(items)
        real = local % n
        start = real * self.batch_size
        return bucket, [items[(start + j) % n] for j in range(self.batch_size)]


# ----------------------------------------------------------------------------- per-image geometry
def cover_size(width: int, height: int, target_w: int, target_h: int, do_upscale: bool = False) -> tuple[int, int]:
    """ObjectCoverResize's output size (transform.py:32-55): the smallest scaling that covers the target
    on both sides, ceil'd; (scaled_w, scaled_h)."""
    if (width < target_w or height < target_h) and not do_upscale:
        raise ValueError(f"Image is too small to crop to {target_w}x{target_h}")
    s = max(target_w / width, target_h / height)
    return math.ceil(width * s), math.ceil(height * s)


def crop_params(scaled_w: int, scaled_h: int, target_w: int, target_h: int,
                generator: torch.Generator | None = None) -> tuple[int, int]:
    """RandomCrop.get_params (torchvision; called at text_to_image.py:164-167): (top, left) drawn with
    torch.randint over the valid offsets, (0, 0) when the sizes already match."""
    if scaled_w == target_w and scaled_h == target_h:
        return 0, 0
    top = int(torch.randint(0, scaled_h - target_h + 1, size=(1,), generator=generator).item())
    left = int(torch.randint(0, scaled_w - target_w + 1, size=(1,), generator=generator).item())
    return top, left


def cover_resize_crop(img_u8: torch.Tensor, target_w: int, target_h: int, out: torch.Tensor, top: int, left: int,
                      scaled: tuple[int, int], workspace: torch.Tensor | None = None) -> torch.Tensor:
    """img_u8: device uint8 [H, W, 3]; out: device fp16 [3, target_h, target_w] (a batch slot)."""
    H, W = int(img_u8.shape[0]), int(img_u8.shape[1])
    sw, sh = scaled
    need = ops.cover_resize_crop_workspace(H, W, sh, sw, top, target_h, target_w)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(need // 4 + 1, dtype=torch.float32, device=img_u8.device)
    ops.cover_resize_crop(img_u8, H, W, sh, sw, top, left, target_h, target_w, workspace, out)
    return out


# ----------------------------------------------------------------------------- loader
class BucketLoader:
    """One bucketed batch per step (get_dataloader_for_bucketing + concatnate_collate_fn semantics):
    batch dict with image fp16 [B,3,h,w] (device), original_size / target_size / crop_coords_top_left
    int64 [B,2] (device; (h, w) of the resized image, of the crop, and (top, left)), and caption list.

    `images[i]` is anything `decode(images[i])` turns into a uint8 [H,W,3] array (default: a PIL path /
    array passthrough); `sizes[i]` = (width, height) as the reference's imagesize scan records.

    Buckets with a side longer than `max_side` px are dropped before images are assigned (SURVEY gotcha
    #8: JiT's RoPE covers rope_axes_lens[1..2] * patch_size = 128 * 16 = 2048 px per side, while
    generate_buckets() also yields e.g. 64 x 16384; the reference would fail in its RoPE gather).

    Data-parallel sharding (`rank`, `world_size`) follows accelerate's prepare_data_loader over the
    reference's DataLoader(batch_size=1, shuffle=True) (src/trainer/common.py:130, src/dataloader.py:68-87):
    every rank draws the SAME shuffled order of bucket batches (same seed), pads it by cycling from its
    start to a multiple of world_size (even_batches), and rank r takes entries r, r + W, r + 2W, ..."""

    def __init__(self, images: Sequence, sizes: Sequence[tuple[int, int]], captions: Sequence[str] | None,
                 batch_size: int, buckets: np.ndarray | None = None, num_repeats: int = 1, shuffle: bool = True,
                 seed: int = 0, device="cuda", decode: Callable | None = None, do_upscale: bool = False,
                 rank: int = 0, world_size: int = 1, max_side: int | None = 2048):
        if not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} outside world_size {world_size}")
        self.images, self.sizes = images, list(sizes)
        self.captions = list(captions) if captions is not None else None
        buckets = buckets if buckets is not None else generate_buckets()
        if max_side is not None:
            buckets = buckets[(buckets <= max_side).all(axis=1)]
        if len(buckets) == 0:
            raise ValueError(f"no bucket with both sides <= {max_side}")
        self.buckets = buckets
        self.rank, self.world_size = rank, world_size
        self.batches = BucketBatches(assign_buckets(self.sizes, self.buckets), batch_size, num_repeats)
        self.batch_size, self.shuffle, self.device = batch_size, shuffle, torch.device(device)
        self.gen = torch.Generator().manual_seed(seed)
        self.decode = decode if decode is not None else _decode_default
        self.do_upscale = do_upscale
        self._ws = None

    def __len__(self) -> int:
        return -(-len(self.batches) // self.world_size)

    def order(self) -> list[int]:
        """This rank's bucket-batch indices for one epoch (advances the shared shuffle generator)."""
        n = len(self.batches)
        order = torch.randperm(n, generator=self.gen).tolist() if self.shuffle else list(range(n))
        if self.world_size > 1:
            pad = -n % self.world_size
            order = order + [order[i % n] for i in range(pad)]
            order = order[self.rank::self.world_size]
        return order

    def __iter__(self):
        for idx in self.order():
            yield self.batch(idx)

    def batch(self, idx: int) -> dict:
        bucket, items = self.batches[idx]
        tw, th = (int(v) for v in self.buckets[bucket])
        B = len(items)
        img = torch.empty(B, 3, th, tw, dtype=torch.float16, device=self.device)
        orig, tgt, crop = [], [], []
        for slot, i in enumerate(items):
            arr = np.ascontiguousarray(self.decode(self.images[i]), dtype=np.uint8)
            H, W = arr.shape[:2]
            sw, sh = cover_size(W, H, tw, th, self.do_upscale)
            top, left = crop_params(sw, sh, tw, th, self.gen)
            dev = torch.from_numpy(arr).to(self.device, non_blocking=True)
            need = ops.cover_resize_crop_workspace(H, W, sh, sw, top, th, tw)
            if self._ws is None or self._ws.numel() * 4 < need:
                self._ws = torch.empty(need // 4 + 1, dtype=torch.float32, device=self.device)
            ops.cover_resize_crop(dev, H, W, sh, sw, top, left, th, tw, self._ws, img[slot])
            orig.append((sh, sw))
            tgt.append((th, tw))
            crop.append((top, left))
        out = {"image": img,
               "original_size": torch.tensor(orig, dtype=torch.long, device=self.device),
               "target_size": torch.tensor(tgt, dtype=torch.long, device=self.device),
               "crop_coords_top_left": torch.tensor(crop, dtype=torch.long, device=self.device)}
        if self.captions is not None:
            out["caption"] = [self.captions[i] for i in items]
        return out


def _decode_default(x):
    if isinstance(x, np.ndarray):
        return x
    from PIL import Image  # host decode (JPEG/PNG/WebP); the transform chain runs on the device
    with Image.open(x) as im:
        return np.asarray(im.convert("RGB"))
