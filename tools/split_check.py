"""Sub-batch lanes (engine.MICRO_SPLIT) against one lane on the micro config (the DDP tests' model): one training step
per setting on identical inputs, B in {2, 4}, with and without the side stream; prints the parameters whose gradients
differ most (relative L2).

  python tools/split_check.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import vpt.engine as E  # noqa: E402
from tests.test_ddp_gpu import _batch, _step, _trainer  # noqa: E402


def run(split, conc, B):
    E.MICRO_SPLIT, E.CONCURRENT_WGRAD, E.MICRO_SPLIT_MIN_ROWS = split, conc, 0
    dev = torch.device("cuda", 0)
    tr, cfg = _trainer(dev)
    _step(tr, _batch(dev), slice(0, B), dev)
    torch.cuda.synchronize()
    return tr.engine.grads.float().clone(), tr.engine.layout


def hook_check(split, B):
    """Copies every bucket's gradient slice at its on_ready call (on the caller's stream, as GradSync's wire cast does)
    and compares the copies with the final gradients."""
    from vpt.ddp import grad_buckets
    E.MICRO_SPLIT, E.CONCURRENT_WGRAD, E.MICRO_SPLIT_MIN_ROWS = split, True, 0
    dev = torch.device("cuda", 0)
    tr, cfg = _trainer(dev)
    buckets = {n: (lo, hi) for n, lo, hi in grad_buckets(tr.engine.layout, cfg.depth)}
    snaps = {}

    def hook(name):
        lo, hi = buckets[name]
        snaps[name] = tr.engine.grads[lo:hi].clone()
    _step(tr, _batch(dev), slice(0, B), dev, on_ready=hook)
    torch.cuda.synchronize()
    bad = {}
    for n, v in snaps.items():
        lo, hi = buckets[n]
        ref = tr.engine.grads[lo:hi]
        if not torch.equal(v, ref):
            bad[n] = float((v - ref).norm() / ref.norm().clamp_min(1e-30))
    print(json.dumps({"hook_check": {"split": split, "B": B, "buckets": sorted(snaps), "stale": bad}}), flush=True)


def main():
    for split in (1, 2):
        for B in (2, 4):
            hook_check(split, B)
    for B in (2, 4):
        for conc in (True, False):
            g1, lay = run(1, conc, B)
            g2, _ = run(2, conc, B)
            rows = []
            for s in lay.specs:
                a, b = g1[s.offset:s.offset + s.numel], g2[s.offset:s.offset + s.numel]
                d = float((a - b).norm() / a.norm().clamp_min(1e-30))
                rows.append((d, s.name))
            rows.sort(reverse=True)
            print(json.dumps({"B": B, "side": conc, "total_rel": float((g1 - g2).norm() / g1.norm()),
                              "worst": [(n, round(d, 6)) for d, n in rows[:6]]}), flush=True)


if __name__ == "__main__":
    main()
