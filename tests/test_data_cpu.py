"""Host logic of the bucketed data path (vpt/data.py) against the oracle restatement and the reference's
golden bucket lists / known answers. CPU only (no kernel calls)."""

import math
import random

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from oracle import data_oracle as DO
from oracle import jit_oracle as O
from vpt import data as D

GOLD = "tests/golden/ops.safetensors"


@pytest.mark.parametrize("args", [(1048576, 1024, 64, 384), (1048576, 1024, 64, 64), (4096, 64, 64, 64),
                                  (65536, 256, 128, 256)])
def test_generate_buckets_vs_reference_fixture(args):
    """generate_buckets == the reference's own output (tests/golden/make_golden.py)."""
    ref = load_file(GOLD)["buckets/" + "_".join(map(str, args))]
    assert torch.equal(torch.from_numpy(D.generate_buckets(*args)).to(ref.dtype), ref)


def test_bucket_counts_known_answer():
    """tests/test_dataset.py:19-44 of the reference: 31 buckets at base 1024 / step 64 / min 64; 1 at 64."""
    assert len(D.generate_buckets(1024 * 1024, 1024, 64, 64)) == 31
    assert len(D.generate_buckets(64 * 64, 64, 64, 64)) == 1


def test_find_nearest_matches_oracle():
    b = D.generate_buckets(1024 * 1024, 1024, 64, 384)
    mgr = D.AspectRatioBucketManager(b)
    blist = [tuple(map(int, x)) for x in b]
    rng = random.Random(0)
    for _ in range(2000):
        w, h = rng.randint(300, 5000), rng.randint(300, 5000)
        try:
            ref = O.find_nearest_bucket(blist, w, h)
        except AssertionError:
            with pytest.raises(AssertionError):
                mgr.find_nearest(w, h)
            continue
        assert mgr.find_nearest(w, h) == ref
        bw, bh = blist[ref]
        assert bw <= w and bh <= h


@pytest.mark.parametrize("bs,rep", [(1, 1), (4, 1), (8, 3), (5, 2)])
def test_bucket_batches_match_reference_indexing(bs, rep):
    rng = random.Random(bs * 10 + rep)
    sizes = [(rng.randint(600, 3000), rng.randint(600, 3000)) for _ in range(300)]
    buckets = D.generate_buckets(1024 * 1024, 1024, 64, 384)
    subsets = D.assign_buckets(sizes, buckets)
    mine = D.BucketBatches(subsets, bs, rep)
    ref = DO.BucketIndex([items for items in subsets.values() if items], bs, rep)
    assert len(mine) == len(ref)
    for i in range(len(ref)):
        b, items = mine[i]
        assert items == ref[i]
        bw, bh = buckets[b]
        assert all(D.AspectRatioBucketManager(buckets).find_nearest(*sizes[j]) == b for j in items)


def test_cover_size_and_crop_params():
    # ObjectCoverResize: smallest scale covering the bucket, ceil'd (transform.py:41-46)
    sw, sh = D.cover_size(2000, 1500, 1152, 896)
    s = max(1152 / 2000, 896 / 1500)
    assert (sw, sh) == (math.ceil(2000 * s), math.ceil(1500 * s)) and sw >= 1152 and sh >= 896
    with pytest.raises(ValueError):
        D.cover_size(1000, 800, 1024, 1024)
    assert D.cover_size(1000, 800, 1024, 1024, do_upscale=True)[1] >= 1024
    # RandomCrop.get_params: randint(0, H-h+1) then randint(0, W-w+1); (0, 0) for an exact fit
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    top, left = D.crop_params(1300, 900, 1152, 896, g1)
    assert top == int(torch.randint(0, 900 - 896 + 1, (1,), generator=g2).item())
    assert left == int(torch.randint(0, 1300 - 1152 + 1, (1,), generator=g2).item())
    assert D.crop_params(1152, 896, 1152, 896) == (0, 0)


def test_oracle_transform_chain_shapes():
    img = np.random.default_rng(0).integers(0, 256, (700, 900, 3), dtype=np.uint8)
    out, (sh, sw) = DO.transform_chain(img, 512, 384, 3, 0)  # cover size (399, 512): top in [0, 15]
    assert (sh, sw) == (399, 512)
    assert out.shape == (3, 384, 512) and out.dtype == torch.float16
    assert out.abs().max() <= 1.3  # bicubic ringing overshoots [-1, 1] on noise


def test_bucket_loader_drops_buckets_beyond_rope_range():
    """SURVEY gotcha #8: generate_buckets() yields sides up to 16384 px; JiT's RoPE covers 2048 px
    per side (rope_axes_lens 128 x patch 16), so the loader keeps only buckets within it."""
    full = D.generate_buckets()
    assert full.max() > 2048
    ld = D.BucketLoader([], [], None, batch_size=1, device="cpu")
    assert ld.buckets.max() <= 2048 and len(ld.buckets) == int((full <= 2048).all(1).sum())
    # an extreme panorama lands in the widest bucket the model can embed
    sizes = [(9000, 600)]
    ld = D.BucketLoader([None], sizes, None, batch_size=1, device="cpu")
    b, _ = ld.batches[0]
    assert ld.buckets[b][0] <= 2048


@pytest.mark.parametrize("world", [2, 3, 4])
def test_bucket_loader_rank_sharding(world):
    """accelerate prepare_data_loader semantics (src/trainer/common.py:130): one shared shuffled order,
    padded by cycling to a multiple of world_size, rank r takes r::world; every batch is seen, ranks
    are disjoint up to the padding, lengths are equal."""
    rng = random.Random(7)
    sizes = [(rng.randint(1100, 2500), rng.randint(1100, 2500)) for _ in range(61)]
    n = len(D.BucketLoader([None] * 61, sizes, None, batch_size=4, device="cpu", seed=3).batches)
    ref = torch.randperm(n, generator=torch.Generator().manual_seed(3)).tolist()
    padded = ref + [ref[i % n] for i in range(-n % world)]
    orders = []
    for r in range(world):
        ld = D.BucketLoader([None] * 61, sizes, None, batch_size=4, device="cpu", seed=3, rank=r, world_size=world)
        o = ld.order()
        assert len(o) == len(ld) == -(-n // world)
        assert o == padded[r::world]
        orders.append(o)
    allx = [i for o in orders for i in o]
    assert sorted(set(allx)) == list(range(n))
    assert len(allx) - n == -n % world  # only the padding repeats
    with pytest.raises(ValueError):
        D.BucketLoader([], [], None, batch_size=1, device="cpu", rank=2, world_size=2)
