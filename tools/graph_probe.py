"""How much of the C3 step is launch overhead: one JiT-B/16 training step (B=8, 1024^2 bucket, fixed t, no CFG drop:
noise + patchify, forward, x-loss, backward, fused RAdamScheduleFree over the flat buffer) timed eagerly (ctypes
launches on torch's current stream) and as a replayed HIP graph (torch.cuda.CUDAGraph capture of the same calls),
events on the stream, medians over rounds. A probe of the dispatch gaps, not a product path: the captured step bakes
in its host scalars (noise seed, optimizer schedule).

  python tools/graph_probe.py [--rounds 5] [--steps 10]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vpt.config import JiT_B_16_Config, JiTTrainingConfig  # noqa: E402
from vpt.jit_train import JiTTrainer  # noqa: E402
from vpt.optim import RAdamScheduleFreeFlat  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--bucket", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = JiTTrainer(JiT_B_16_Config(), bench.N_CLASSES, JiTTrainingConfig(loss_target="image"), device=dev, seed=1)
    tr.engine.init_weights(seed=0)
    opt = RAdamScheduleFreeFlat(tr.engine.params, tr.engine.grads, lr=1e-4)
    opt.train()
    b = bench.make_batches(8, dev, seed=100)[args.bucket]
    t_fixed = torch.full((8,), 0.5, device=dev)
    s = opt.begin_step()
    nparam = tr.engine.params.numel()

    def step():
        tr.step(b["images"], b["ids"], b["mask"], b["original_size"], b["target_size"], b["crop_coords"], t=t_fixed,
                drop_context=False)
        opt.apply_range(s, 0, nparam)

    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record(cur)
        for _ in range(args.steps):
            fn()
        e1.record(cur)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    res = {"eager": [], "graph": []}
    for r in range(args.rounds):
        for k in (("eager", "graph") if r % 2 == 0 else ("graph", "eager")):
            res[k].append(timed(step if k == "eager" else g.replay))
    med = {k: round(statistics.median(v), 3) for k, v in res.items()}
    print(json.dumps({"ms_per_step": med, "graph_vs_eager": round(med["graph"] / med["eager"], 4),
                      "bucket_wh": [b["W"], b["H"]], "nodes": None}), flush=True)


if __name__ == "__main__":
    main()
