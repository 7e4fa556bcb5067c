"""Repeated-run determinism stress of the production multi-stream schedule: the flat gradient after 3 accumulating
steps (depth-4 JiT-B/16 blocks, context from block 2, B=4 512x448, a padded context row) on the production streams
(side-stream weight gradients, forward lanes) against the single-stream schedule, `--repeats` fresh trainers; any
parameter whose gradient differs bitwise is reported with its relative difference.

  python tools/determinism_stress.py [--repeats 10] [--split 1]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

import vpt.engine as E  # noqa: E402
from vpt.config import JiT_B_16_Config, JiTTrainingConfig  # noqa: E402
from vpt.jit_train import JiTTrainer  # noqa: E402


def run(conc: bool, split: int):
    E.CONCURRENT_WGRAD, E.MICRO_SPLIT = conc, split
    cfg = JiT_B_16_Config(depth=4, context_start_block=2)
    tr = JiTTrainer(cfg, 100, JiTTrainingConfig(loss_target="image"), device="cuda", seed=3)
    tr.engine.init_weights(seed=0)
    g = torch.Generator().manual_seed(4)
    out = []
    for step in range(3):
        img = (torch.rand(4, 3, 512, 448, generator=g) * 2 - 1).half().cuda()
        ids = torch.randint(0, 100, (4, 16), generator=g)
        mask = torch.ones(4, 16, dtype=torch.long)
        mask[1, 9:] = 0
        size = torch.tensor([[512, 448]] * 4, device="cuda")
        tr.step(img, ids, mask, size, size.clone(), torch.zeros(4, 2, dtype=torch.long, device="cuda"),
                t=torch.tensor([0.3, 0.8, 0.5, 0.1]), drop_context=False, accumulate=step > 0)
        torch.cuda.synchronize()
        out.append(tr.engine.grads.clone())
    return out, tr.engine.layout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=10)
    ap.add_argument("--split", type=int, default=None, help="forward lanes (default: the engine's MICRO_SPLIT)")
    args = ap.parse_args()
    defaults = (E.CONCURRENT_WGRAD, E.MICRO_SPLIT if args.split is None else args.split)
    ref, lay = run(False, 1)
    bad = []
    for r in range(args.repeats):
        got, _ = run(*defaults)
        for st in range(3):
            a, b = ref[st], got[st]
            for s in lay.specs:
                x, y = a[s.offset:s.offset + s.numel], b[s.offset:s.offset + s.numel]
                if not torch.equal(x, y):
                    bad.append((r, st, s.name, ((x - y).norm() / x.norm().clamp_min(1e-30)).item()))
        print(f"repeat {r}: {sum(1 for x in bad if x[0] == r)} differing (step, parameter) pairs", flush=True)
    print(json.dumps({"repeats": args.repeats, "schedule": {"concurrent_wgrad": defaults[0], "micro_split": defaults[1]},
                      "differing": len(bad), "first": bad[:20]}))


if __name__ == "__main__":
    main()
