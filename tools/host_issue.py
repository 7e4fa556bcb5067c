"""Host issue time of the C3 training step against its GPU time: K steps issued back to back (no synchronisation
inside), the host clock read after the issue loop and again after torch.cuda.synchronize(). When the issue time
approaches the GPU time, the step is launch-bound (host) rather than kernel-bound.

  python tools/host_issue.py [--steps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)
os.environ["GPU_MAX_HW_QUEUES"] = "8"

import torch  # noqa: E402

import bench  # noqa: E402
from vpt.config import JiT_B_16_Config, JiTTrainingConfig  # noqa: E402
from vpt.jit_train import JiTTrainer  # noqa: E402
from vpt.optim import RAdamScheduleFreeFlat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = JiTTrainer(JiT_B_16_Config(), bench.N_CLASSES, JiTTrainingConfig(loss_target="image"), device=dev, seed=1)
    tr.engine.init_weights(seed=0)
    opt = RAdamScheduleFreeFlat(tr.engine.params, tr.engine.grads, lr=1e-4)
    opt.train()
    batches = bench.make_batches(8, dev, seed=100)

    def step(i):
        b = batches[i % len(batches)]
        tr.step(b["images"], b["ids"], b["mask"], b["original_size"], b["target_size"], b["crop_coords"])
        opt.step()

    for i in range(2 * len(batches)):
        step(i)
    torch.cuda.synchronize()
    res = {}
    for name, k in (("one_step", 1), ("k_steps", args.steps)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            step(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[name] = {"issue_ms_per_step": round((t1 - t0) / k * 1e3, 3), "wall_ms_per_step": round((t2 - t0) / k * 1e3, 3)}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
