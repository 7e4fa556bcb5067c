"""Is the C5 step host-bound? Host enqueue time of each step (no sync) against the synced wall time per step, on the
bench's C5 workload (bench.py bench_c5: B = 4, the 5 SDXL buckets in the bench's order).
    python tools/c5_host_probe.py [--steps 10]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vision-pt_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from vpt.sdxl_flow import SDXL_BUCKETS_5, SDXLFlowMatchQLoRA
    torch.cuda.set_device(0)
    m = SDXLFlowMatchQLoRA(B=4, device="cuda", seed=0)
    batches = [m.make_inputs(seed=1 + i, latent=(H // 8, W // 8)) for i, (W, H) in enumerate(SDXL_BUCKETS_5)]
    for i in range(len(batches)):
        m.step(*batches[i])
    torch.cuda.synchronize()
    # (1) synced per step: wall of one step, host enqueue part of it
    enq, wall = [], []
    for i in range(a.steps):
        t0 = time.perf_counter()
        m.step(*batches[i % len(batches)])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    # (2) back to back: host time to enqueue all steps, then the drain
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        m.step(*batches[i % len(batches)])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(json.dumps({"synced_enqueue_ms": [round(x, 2) for x in enq], "synced_wall_ms": [round(x, 2) for x in wall],
                      "b2b_enqueue_ms_per_step": round((t1 - t0) * 1e3 / a.steps, 2),
                      "b2b_wall_ms_per_step": round((t2 - t0) * 1e3 / a.steps, 2),
                      "b2b_drain_ms": round((t2 - t1) * 1e3, 2)}))


if __name__ == "__main__":
    main()
