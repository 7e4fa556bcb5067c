"""CPU oracle for the bucketed-batch data path. TEST INFRASTRUCTURE ONLY:
imported by tests/ (never by vpt); it is the checker, not the thing measured or shipped.

Restated from the reference (file:line) with plain torch / numpy:
  - per-image transform chain, src/dataset/text_to_image.py:145-158 (PILToTensor -> ToDtype(float16,
    scale=True) -> Normalize(0.5, 0.5) -> ObjectCoverResize) and :164-177 (RandomCrop), with
    ObjectCoverResize from src/dataset/transform.py:32-55. torchvision is not installed here; its v2
    functional ops used by that chain are thin wrappers, restated as: to_dtype = `.to(fp16).mul_(1/255)`,
    normalize = `.sub_(mean).div_(std)` with fp16 mean/std, resize of a non-float32 float image = cast to
    float32, torch.nn.functional.interpolate(mode="bicubic", antialias=True, align_corners=False) (the
    ATen kernel torchvision dispatches to), cast back; crop = slicing.
  - bucket dataset indexing, src/dataset/bucket.py:45-121 (Bucket.to_local_idx / __getitem__,
    BucketDataset.__len__ / __getitem__) over torch.utils.data.ConcatDataset (text_to_image.py:508-512),
    restated because the module imports torchvision.
Parity pinning: the resize/normalise arithmetic IS torch's own CPU kernel; the torchvision wrapper
semantics above are restated, not executed (parity of that glue is unpinned beyond this restatement).
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def transform_chain(img_u8_hwc: np.ndarray, target_w: int, target_h: int, top: int, left: int,
                    do_upscale: bool = False) -> tuple[torch.Tensor, tuple[int, int]]:
    """fp16 [3, target_h, target_w] crop and the resized (h, w), as the reference's TextToImageBucket
    produces for one image with crop offsets (top, left)."""
    x = torch.from_numpy(np.ascontiguousarray(img_u8_hwc)).permute(2, 0, 1).contiguous()  # PILToTensor: CHW
    x = x.to(torch.float16).mul_(1.0 / 255)                                                # ToDtype(scale=True)
    mean = torch.as_tensor([0.5, 0.5, 0.5], dtype=torch.float16).view(-1, 1, 1)
    std = torch.as_tensor([0.5, 0.5, 0.5], dtype=torch.float16).view(-1, 1, 1)
    x = x.sub_(mean).div_(std)                                                             # Normalize
    h, w = x.shape[1], x.shape[2]
    if (w < target_w or h < target_h) and not do_upscale:
        raise ValueError("Image is too small")
    s = max(target_w / w, target_h / h)
    sw, sh = math.ceil(w * s), math.ceil(h * s)
    if (sh, sw) != (h, w):
        y = F.interpolate(x.float()[None], size=[sh, sw], mode="bicubic", align_corners=False, antialias=True)[0]
        x = y.to(torch.float16)
    return x[:, top:top + target_h, left:left + target_w].contiguous(), (sh, sw)


class BucketIndex:
    """ConcatDataset([BucketDataset(Bucket(items, bs, repeats))]) restated (bucket.py:45-121)."""

    def __init__(self, subsets: list[list[int]], batch_size: int, num_repeats: int = 1):
        self.subsets, self.bs, self.rep = subsets, batch_size, num_repeats

    def __len__(self):
        return sum(math.ceil(len(s) * self.rep / self.bs) for s in self.subsets)

    def __getitem__(self, idx: int) -> list[int]:
        for items in self.subsets:
            n_samples = math.ceil(len(items) * self.rep / self.bs)  # BucketDataset.num_samples
            if idx < n_samples:
                real_idx = idx % len(items)                          # BucketDataset.__getitem__
                start, stop = real_idx * self.bs, real_idx * self.bs + self.bs
                local = (np.arange(start, stop) % len(items)).tolist()  # Bucket.to_local_idx(slice)
                return [items[i] for i in local]
            idx -= n_samples
        raise IndexError(idx)
