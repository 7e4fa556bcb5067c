#!/usr/bin/env python3
"""Training-throughput benchmark: JiT-B/16 rectified-flow training step at 1024^2 with aspect-ratio
bucketing (BASELINE.json config 3; config 4 when launched with N>1 ranks).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

One step per rank = one batch of B=8 images of one bucket (5 buckets {1024x1024, 960x1088,
1088x960, 896x1152, 1152x896}; each epoch's bucket batches in one seeded shuffled order shared by all ranks,
rank r taking entries r, r+N, ... as accelerate's prepare_data_loader does): noise + patchify, JiT forward,
x-loss, backward, RCCL all-reduce of the gradients (N>1: bf16 wire, per-block buckets launched as the
backward completes them), fused RAdamScheduleFree step per bucket on a side stream as each reduction lands
— no work skipped. `--workload c2`: BASELINE config 2 (512^2, B=16); `--workload c5`: config 5. Synthetic data resident in HBM (no decoder), random-init
weights of the JiT_B_16_Config architecture, class-conditional context (V=10,000, 64 tokens, valid
length U[8,64], CFG drop p=0.1). Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

# HIP hardware queues per process (read at HIP's initialisation, so set before torch loads). 4 (HIP's own default): with
# the collectives really running in the step (--force-collective, r06g, one box, 3 interleaved repeats) 8 queues cost
# 16 % (152.8-153.8 vs 179.3-181.5 img/s at 4; 2 queues 181.0-181.2), while without them 4 and 8 are level (182.2-183.0)
# and 2 lose 8.5 %. --hw-queues N sets it (<= 32); without the flag an exported GPU_MAX_HW_QUEUES is kept, else 4. The
# bench line records the REQUESTED value (`hw_queues_requested`): under a profiler that initialises the HIP runtime
# first, the runtime may have read the variable before this line.
if "--hw-queues" in sys.argv:
    _hwq = int(sys.argv[sys.argv.index("--hw-queues") + 1])
    if not 1 <= _hwq <= 32:
        raise SystemExit("--hw-queues: 1..32")
    os.environ["GPU_MAX_HW_QUEUES"] = str(_hwq)
else:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "4")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train images/sec (whole node), JiT 1024² bucketed, 1/2/4/8 MI355X"
METRIC_C2 = "train images/sec, JiT-B/16 512² single-bucket, 1 MI355X"
BUCKETS = [(1024, 1024), (960, 1088), (1088, 960), (896, 1152), (1152, 896)]  # (W, H)
BUCKETS_C2 = [(512, 512)]
N_CLASSES = 10_000
N_CTX = 64
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBS = 8000.0


def measured_traffic(op: str, workload: str = "c3"):
    """HBM bytes per launch of `op` from the committed rocprofv3 PMC summary of this workload
    (profiles/traffic_latest.json = the c3 headline; profiles/traffic_<workload>.json otherwise;
    tools/round_profile.sh -> tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE passes, gfx950 read
    correction), or None when no summary of this workload is committed."""
    name = "traffic_latest.json" if workload == "c3" else f"traffic_{workload}.json"
    path = os.path.join(ROOT, "profiles", name)
    try:
        d = json.load(open(path))
        return d[op]["hbm_bytes_per_launch"], f"profiles/{name} ({d.get('_tag', '?')})"
    except (OSError, KeyError, ValueError):
        return None, None


def shared_order(n_buckets: int, steps: int, world: int, rank: int, seed: int = 7) -> list[int]:
    """Per-step bucket index of this rank: accelerate's prepare_data_loader over a shuffled bucket-batch list
    (vpt.data.BucketLoader.order): every rank draws the SAME seeded permutation of each epoch's bucket batches
    (n_buckets per rank per epoch) and takes entries rank, rank + world, ... -- so ranks hold DIFFERENT
    buckets in the same step (the 4032-4170-token skew is inside the timed region, as in training)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    while len(out) < steps:
        epoch = [i % n_buckets for i in range(n_buckets * world)]
        perm = torch.randperm(len(epoch), generator=g).tolist()
        out += [epoch[perm[j]] for j in range(rank, len(epoch), world)]
    return out[:steps]


def train_flops_per_image(np_: int, D=768, F=2048, depth=12, cs=4, bd=128) -> float:
    """3x forward matmul FLOPs + 3x attention forward (no recompute credit)."""
    f = 2 * np_ * (768 * bd + bd * D)
    for l in range(depth):
        n = np_ + 10 + (64 if l >= cs else 0)
        f += 2 * n * (4 * D * D + 3 * D * F) + 4 * n * n * D
    f += 2 * np_ * (3 * D * F + D * 768)
    return 3.0 * f


def make_batches(B: int, device, seed: int, buckets=BUCKETS):
    g = torch.Generator(device="cpu").manual_seed(seed)
    out = []
    for (W, H) in buckets:
        img = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).half().to(device)
        lens = torch.randint(8, N_CTX + 1, (B,), generator=g)
        ids = torch.randint(0, N_CLASSES, (B, N_CTX), generator=g)
        mask = (torch.arange(N_CTX)[None, :] < lens[:, None]).long()
        ids = torch.where(mask.bool(), ids, torch.full_like(ids, N_CLASSES))
        size = torch.tensor([[H, W]]).repeat(B, 1).to(device)
        out.append(dict(images=img, ids=ids.to(device), mask=mask.to(device), original_size=size,
                        target_size=size.clone(), crop_coords=torch.zeros(B, 2, dtype=torch.long, device=device),
                        W=W, H=H))
    return out


def _cpu_leg(oc, B: int, buckets, n_classes: int, steps: int, budget_s: float):
    """One CPU-oracle leg: 1 warm-up step, then up to `steps` timed steps (stopping early past budget_s) of the
    fp32 restatement's training step (forward, x-loss, backward, AdamW: schedulefree is not installed)."""
    from oracle import jit_oracle as O
    model = O.OracleJiT(oc)
    emb = torch.nn.Parameter(torch.randn(n_classes + 1, oc.hidden_size) * 0.02)
    opt = torch.optim.AdamW(list(model.parameters()) + [emb], lr=1e-4)
    g = torch.Generator().manual_seed(0)

    def one(W, H):
        batch = dict(image=(torch.rand(B, 3, H, W, generator=g) * 2 - 1).half(),
                     noise=torch.randn(B, 3, H, W, generator=g).half(),
                     t=(torch.randn(B, generator=g) * 0.8 - 0.8).sigmoid(),
                     ids=torch.randint(0, n_classes, (B, N_CTX), generator=g),
                     mask=torch.ones(B, N_CTX, dtype=torch.long),
                     original_size=torch.tensor([[H, W]] * B), target_size=torch.tensor([[H, W]] * B),
                     crop_coords=torch.zeros(B, 2, dtype=torch.long))
        loss, _ = O.train_step_loss(model, emb, batch, "image")
        loss.backward()
        opt.step()
        opt.zero_grad()

    one(*buckets[0])  # warm-up at the sample's own size (allocator, threads)
    n, t0 = 0, time.perf_counter()
    while n < steps:
        W, H = buckets[n % len(buckets)]
        one(W, H)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return n, dt


def cpu_baseline(workload: str = "c3"):
    """Times the CPU oracle (oracle/jit_oracle.py, a parity-pinned fp32 restatement of the reference step; AdamW
    stands in for schedulefree, which is not installed) on the host cores, BASELINE.md §4.3's three legs: C1 (JiT
    tiny 256^2, B=4), JiT-B/16 512^2 B=1 and JiT-B/16 at the 1024^2-area buckets B=1, each 1 warm-up + 3 timed steps.
    `value` is the leg of the benched workload (c3: the 1024^2 buckets; c2: 512^2), in img/s."""
    from oracle import jit_oracle as O
    from tests.golden import golden_configs as GC
    threads = torch.get_num_threads()
    legs = {}
    for name, oc, B, bk, ncls, budget in (("c1_tiny_256sq_b4", GC.c1_config(), 4, [(256, 256)], 1000, 10.0),
                                          ("jit_b16_512sq_b1", O.jit_b16(), 1, BUCKETS_C2, N_CLASSES, 10.0),
                                          ("jit_b16_1024area_b1", O.jit_b16(), 1, BUCKETS, N_CLASSES, 25.0)):
        n, dt = _cpu_leg(oc, B, bk, ncls, steps=3, budget_s=budget)
        legs[name] = dict(value=round(n * B / dt, 5), unit="img/s", steps=n, seconds=round(dt, 2), batch=B,
                          buckets_wh=bk)
    main = legs["jit_b16_512sq_b1" if workload == "c2" else "jit_b16_1024area_b1"]
    area = "512^2" if workload == "c2" else "1024^2-area buckets"
    return dict(value=main["value"], unit="img/s", cores=threads, kind="port",
                sample=f"{main['steps']} JiT-B/16 training steps (B=1, {area}, fp32, AdamW) on the CPU oracle after 1 "
                       f"warm-up, {main['seconds']} s, torch threads={threads}; legs = BASELINE.md §4.3's C1 / 512^2 / "
                       f"1024^2 samples",
                legs=legs)


def roofline_entry(name: str, st: dict, workload: str = "c3"):
    """MFMA roofline of one probed kernel: algorithmic FLOPs / mean launch time vs the bf16 peak, with the PMC
    HBM bytes per launch (profiles/traffic_*.json) against the launch's compulsory bytes."""
    traffic, src = measured_traffic(name, workload)
    comp = st["mean_compulsory_bytes"]
    return {"bound": "mfma", "kernel": name, "achieved": round(st["tflops"], 2), "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s", "frac": round(st["tflops"] / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
            "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": src,
            "compulsory_bytes_per_launch": round(comp), "traffic_over_compulsory":
                round(traffic / comp, 2) if (traffic and comp) else None,
            "algorithmic_gflop_per_launch": round(st["mean_gflop"], 3), "mean_launch_ms": round(st["mean_ms"], 4),
            "launches_probed": st["launches"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)    # >= 10 warm-up, >= 50 timed steps
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: 8 for c3, 16 for c2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--breakdown", default=None, help="write per-shape GEMM probe totals (JSON) to this file")
    ap.add_argument("--grad-ckpt", action="store_true",
                    help="gradient checkpointing on (denoiser.py:945-967): keep block inputs, recompute in backward")
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="optimizer per gradient bucket on a side stream as each all-reduce lands (auto: off -- "
                         "with the RCCL all-reduces really in the step (--force-collective, r06f, 4 HW queues) on "
                         "177.2 / 177.5 vs off 177.8 / 177.7 img/s; the all-reduces themselves run under the backward "
                         "at any setting)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (applied at import; default: the exported value, else 4)")
    ap.add_argument("--force-collective", action="store_true",
                    help="world 1 only: initialise a one-rank nccl (RCCL) group and run every gradient bucket's "
                         "all-reduce (bf16 wire cast included) and the loss all-reduce inside the timed step, as at "
                         "N > 1 -- to measure the N > 1 schedule (overlap, HW queues) with the collectives really "
                         "running on one GPU")
    ap.add_argument("--streams", default="multi", choices=["multi", "single"],
                    help="multi: the engine's concurrent streams (the backward's weight-gradient GEMMs beside the "
                         "input-gradient chain, vpt.engine.CONCURRENT_WGRAD: +2.2 %% per C3 step, r05v; the blocks as "
                         "sub-batch lanes, vpt.engine.MICRO_SPLIT); single: every kernel on the step's stream. The probe "
                         "pass always runs single, so per-kernel times are not shared with a concurrent kernel")
    ap.add_argument("--workload", default="c3", choices=["c2", "c3", "c5"],
                    help="c3: JiT-B/16 1024^2 bucketed (the headline); c2: JiT-B/16 512^2 B=16; "
                         "c5: SDXL QLoRA transformer stacks")
    args = ap.parse_args()
    if args.workload == "c5":
        return bench_c5(args)
    c2 = args.workload == "c2"
    buckets = BUCKETS_C2 if c2 else BUCKETS
    if args.batch is None:
        args.batch = 16 if c2 else 8

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VPT_DIST_BACKEND=gloo: a rehearsal of the N > 1 path with several ranks sharing the box's GPUs (RCCL needs
    # one GPU per rank); the measured line is always nccl (= RCCL over xGMI), one rank per GPU
    backend = os.environ.get("VPT_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    force = bool(args.force_collective)
    if force and world > 1:
        raise SystemExit("--force-collective is the world-1 stand-in for N > 1")
    if world > 1 or force:
        if force:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # RCCL prints its version banner on stdout when it creates the communicator; the driver reads rank 0's stdout as
        # ONE JSON line, so stdout goes to stderr while the group (and its communicator, by the barrier) is created
        saved = os.dup(1)
        sys.stdout.flush()
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend, device_id=device if backend == "nccl" else None)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    from vpt import engine as vpt_engine
    from vpt import ops
    from vpt.config import JiT_B_16_Config, JiTTrainingConfig
    from vpt.ddp import GradSync, LossLog, grad_buckets
    from vpt.jit_train import JiTTrainer
    from vpt.optim import RAdamScheduleFreeFlat

    if args.streams == "single":
        vpt_engine.CONCURRENT_WGRAD = False
        vpt_engine.MICRO_SPLIT = 1
    timed_streams = dict(wgrad_stream="side" if vpt_engine.CONCURRENT_WGRAD else "step",
                         sub_batches=vpt_engine.MICRO_SPLIT, hw_queues_requested=int(os.environ["GPU_MAX_HW_QUEUES"]))
    cfg = JiT_B_16_Config()
    trainer = JiTTrainer(cfg, N_CLASSES, JiTTrainingConfig(loss_target="image"), device=device, seed=1234 + rank)
    trainer.engine.init_weights(seed=0)  # identical on every rank (replaces DDP's broadcast)
    trainer.engine.set_gradient_checkpointing(args.grad_ckpt)
    opt = RAdamScheduleFreeFlat(trainer.engine.params, trainer.engine.grads, lr=1e-4)
    opt.train()
    # per-block buckets: all-reduced (bf16 wire, as the reference's DDP reduces its bf16 .grad tensors) the
    # moment the backward completes them and stepped by the optimizer on a side stream as each reduction lands
    overlap = args.overlap == "on"
    sync = GradSync(trainer.engine.grads, grad_buckets(trainer.engine.layout, cfg.depth), wire="bf16",
                    overlap=overlap, force_collective=force)
    losslog = LossLog(device, force_collective=force)
    batches = make_batches(args.batch, device, seed=100 + rank, buckets=buckets)
    n_probe = len(buckets)
    order = shared_order(len(buckets), args.warmup + args.steps + n_probe, world, rank)

    def step(i):
        b = batches[order[i]]
        s = opt.begin_step()
        sync.arm(lambda lo, hi, sc, g, **kw: opt.apply_range(s, lo, hi, sc, g, **kw))
        trainer.step(b["images"], b["ids"], b["mask"], b["original_size"], b["target_size"], b["crop_coords"],
                     on_ready=sync.launch)
        sync.launch_rest()
        sync.finish()
        opt.end_step(s)
        losslog.push(trainer._loss)  # the reference's per-step loss gather (2-float all-reduce, read later)

    for i in range(args.warmup):
        step(i)
    # ---- timed region: exactly K steps, no instrumentation
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    loss = None
    while losslog.pending:
        loss = losslog.pop()  # the last timed step's loss, averaged over ranks

    # ---- probe pass (after the timed region): one round of the buckets with HIP events around every
    # launch of the MFMA ops (algorithmic FLOPs) and the memory-bound ops (algorithmic HBM bytes); the weight gradients
    # on the step's stream here, so no kernel's time is shared with a concurrent one
    vpt_engine.CONCURRENT_WGRAD = False
    vpt_engine.MICRO_SPLIT = 1
    mfma_ops = ("attn_fwd", "attn_bwd", "gemm")
    hbm_ops = ("rmsnorm_fwd", "rmsnorm_bwd", "qknorm_rope_fwd", "qknorm_rope_bwd", "patchify",
               "flow_loss", "radam_sf_step")
    probes = {k: ops.KernelProbe(k) for k in mfma_ops + hbm_ops}
    ops.PROBES.update(probes)
    for p in probes.values():
        p.active = True
    for i in range(args.warmup + args.steps, args.warmup + args.steps + n_probe):
        step(i)
    torch.cuda.synchronize()
    for p in probes.values():
        p.active = False
    ops.PROBES.clear()

    imgs = args.batch * args.steps * world
    value = imgs / dt
    stats, hbm = {}, {}
    for k in mfma_ops:
        n, ms, fl = probes[k].summary()
        stats[k] = dict(launches=n, mean_ms=ms, total_ms=n * ms, tflops=(fl / (ms * 1e-3) / 1e12) if ms else 0.0,
                        mean_gflop=fl / 1e9, mean_compulsory_bytes=probes[k].mean_bytes())
    for k in hbm_ops:
        n, ms, nb = probes[k].summary()
        gbs = nb / (ms * 1e-3) / 1e9 if ms else 0.0
        hbm[k] = dict(launches=n, mean_ms=round(ms, 4), mean_mb=round(nb / 1e6, 3), gb_s=round(gbs, 1),
                      frac=round(gbs / PEAK_HBM_GBS, 3))
    gemm_keys = probes["gemm"].by_key()
    if args.breakdown and rank == 0:
        rows = {k: dict(launches=n, ms_per_step=round(t / n_probe, 4), tflops=round(w / (t * 1e-3) / 1e12, 1))
                for k, (n, t, w) in gemm_keys.items()}
        rows = dict(sorted(rows.items(), key=lambda kv: -kv[1]["ms_per_step"]))
        json.dump(rows, open(args.breakdown, "w"), indent=1)
    # headline roofline = the single kernel with the largest time per step: attn_fwd / attn_bwd are one kernel
    # each; the GEMMs are compared shape by shape (the largest GEMM shape's total); the others sit beside it
    single = {k: stats[k]["total_ms"] for k in ("attn_fwd", "attn_bwd")}
    single["gemm"] = max((t for _, t, _ in gemm_keys.values()), default=0.0)
    dom = max(single, key=single.get)
    np_avg = sum((W // 16) * (H // 16) for W, H in buckets) / len(buckets)
    step_tflop = train_flops_per_image(np_avg) * args.batch / 1e12
    wl = ("JiT-B/16 (JiT_B_16_Config) training step, 512^2 single bucket (BASELINE config 2)" if c2 else
          "JiT-B/16 (JiT_B_16_Config) training step, 1024^2 area, 5 aspect-ratio buckets, rank-interleaved "
          "shared shuffled order")
    result = {
        "metric": METRIC_C2 if c2 else METRIC, "value": round(value, 3), "unit": "img/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (HBM-resident, random-init weights)",
        "config": {"workload": wl, "model": "JiT-B/16", "per_gpu_batch": args.batch, "global_batch": args.batch * world,
                   "seq_len": "1034-1098 tokens" if c2 else "4042-4170 tokens", "buckets_wh": buckets,
                   "parallelism": f"dp{world}", "loss_target": "image", "optimizer": "RAdamScheduleFree (fused HIP)",
                   "optimizer_overlap": "per bucket on a side stream during backward" if overlap else
                   "one launch after the backward",
                   "grad_allreduce": ("bf16 wire, per-block buckets overlapped with backward" if world > 1 else
                                      "forced at world 1 (RCCL all-reduces in the step)" if force else None),
                   "grad_checkpointing": bool(args.grad_ckpt),
                   "streams": timed_streams},
        "roofline": roofline_entry(dom, stats[dom], args.workload),
        "roofline_others": {k: roofline_entry(k, stats[k], args.workload) for k in mfma_ops if k != dom},
        "kernels": {k: {kk: round(vv, 4) for kk, vv in v.items()} for k, v in stats.items()},
        "hbm_kernels": hbm,
        "probe_pass": f"{n_probe} steps after the timed region, HIP events on the launching stream, weight gradients "
                      "on the step's stream",
        "model_tflops_per_gpu": round(step_tflop * args.steps / (dt), 2),
        "mfu": round(step_tflop * args.steps / dt / PEAK_BF16_TFLOPS, 4),
        "final_loss": round(loss, 5),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.workload)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1 or force:
        dist.barrier()
        dist.destroy_process_group()


def bench_c5(args):
    """BASELINE config 5 on one GPU: the SDXL flow-matching QLoRA step (train/sdxl/flow_match.py:109-174) on the
    reference's aspect-ratio buckets (configs/sdxl/flow_match/config.yml:46-50: base 1024, step 128, min 384; the
    five nearest to square, 896x1152 ... 1408x768, latents / 8), batch 4, drawn per step from one seeded shuffled
    order: t ~ scale_shift_sigmoid, noising, the UNet's 11 SpatialTransformers (70 blocks, 700 LoRA r=16 targets over
    NF4 bases, dequantised per call as bitsandbytes' MatMul4Bit does -- vpt.sdxl.BASE_MODES) inside a frozen skeleton
    of the UNet's topology (its ResNet / conv path is outside SURVEY §8), velocity MSE, backward, RAdamScheduleFree on
    the adapters (vpt/sdxl_flow.py)."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--workload c5 is a 1-GPU configuration")
    torch.cuda.set_device(0)
    from vpt import ops
    from vpt.sdxl import DEFAULT_BASE_MODE
    from vpt.sdxl_flow import SDXL_BUCKETS_5, SDXLFlowMatchQLoRA
    B = 4
    m = SDXLFlowMatchQLoRA(B=B, device="cuda", seed=0)
    batches = [m.make_inputs(seed=1 + i, latent=(H // 8, W // 8)) for i, (W, H) in enumerate(SDXL_BUCKETS_5)]
    nb = len(batches)
    order = shared_order(nb, args.warmup + args.steps + nb, 1, 0, seed=11)
    for i in range(args.warmup):
        m.step(*batches[order[i]])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        m.step(*batches[order[i]])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loss = m.loss.item()
    # probe pass after the timed region (one step per bucket): GEMM and attention launches timed with HIP events
    probes = {k: ops.KernelProbe(k) for k in ("gemm_lora", "gemm_nf4", "attn_fwd", "attn_bwd", "gemm", "nf4_dequant")}
    ops.PROBES.update(probes)
    for p in probes.values():
        p.active = True
    for i in range(nb):
        m.step(*batches[i])
    torch.cuda.synchronize()
    for p in probes.values():
        p.active = False
    ops.PROBES.clear()
    kern = {}
    for k, pr in probes.items():
        n, ms, fl = pr.summary()
        n_step = n / nb
        if k == "nf4_dequant":  # HBM-bound: algorithmic bytes / time
            kern[k] = dict(launches_per_step=n_step, mean_ms=round(ms, 4), ms_per_step=round(n_step * ms, 3),
                           gb_s=round(fl / (ms * 1e-3) / 1e9, 1) if ms else 0.0,
                           frac=round(fl / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 3) if ms else 0.0)
        else:
            kern[k] = dict(launches_per_step=n_step, mean_ms=round(ms, 4), ms_per_step=round(n_step * ms, 3),
                           tflops=round(fl / (ms * 1e-3) / 1e12, 2) if ms else 0.0)
    if args.breakdown:  # per-shape totals of the base+LoRA GEMMs over the probed steps
        rows = {k: dict(launches=n, total_ms=round(t, 3), tflops=round(w / (t * 1e-3) / 1e12, 1))
                for k, (n, t, w) in sorted(probes["gemm_lora"].by_key().items(), key=lambda kv: -kv[1][1])}
        json.dump(rows, open(args.breakdown, "w"), indent=1)
    # headline roofline: the MFMA op with the largest total time in the step
    dom = max((k for k in kern if k != "nf4_dequant"), key=lambda k: kern[k]["ms_per_step"])
    n, ms, fl = probes[dom].summary()
    tf = fl / (ms * 1e-3) / 1e12 if ms else 0.0
    traffic, tsrc = measured_traffic(dom, "c5")
    if traffic is None:
        # the FETCH_SIZE pass of this command completes, but its WRITE_SIZE pass stalls under rocprofv3 right after
        # HSA init, reproducibly (profiles/r04/r04k_c5_write_size_stall.log), so no read+write figure exists
        tsrc = "unmeasured: rocprofv3 --pmc WRITE_SIZE stalls on the C5 command (profiles/r04/r04k_c5_write_size_stall.log)"
    step_tf = sum(m.flops_per_step((H // 8, W // 8)) for (W, H) in SDXL_BUCKETS_5) / nb / 1e12
    res = {
        "metric": "train images/sec, SDXL QLoRA r=16 flow-matching step (1024^2 bucketed, 5 buckets), 1 MI355X",
        "value": round(B * args.steps / dt, 3), "unit": "img/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16 (NF4 weights)", "data": "synthetic latents / text context / pooled output, random-init weights",
        "config": {"workload": "BASELINE config 5: t ~ scale_shift_sigmoid(-0.8, 0.8), z = t x + (1 - t) eps, "
                               "v = UNet(z, 1000 t, ctx 231x2048, pooled, sizes), loss = mse(v, eps - x); the UNet's "
                               "11 SpatialTransformers (70 blocks, 700 LoRA targets) with the reference's "
                               "conditioning path, its ResNet / conv / resample path replaced by frozen "
                               "pixel-(un)shuffle + Linear maps (outside SURVEY §8, calibrated to unit-RMS outputs); "
                               "VAE and text encoders not run",
                   "buckets_wh": SDXL_BUCKETS_5, "bucket_rule": "base 1024, step 128, min 384 (config.yml:46-50); "
                   "the five nearest to square, one seeded shuffled order",
                   "global_batch": B, "lora_rank": 16, "lora_alpha": 1.0, "adapter_params": m.n_adapter_params(),
                   "loss": "flow-matching velocity MSE (loss_with_predicted_velocity)",
                   "nf4_base": DEFAULT_BASE_MODE, "optimizer": "RAdamScheduleFree (fused HIP)"},
        "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(tf, 2), "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                     "traffic_source": tsrc, "mean_launch_ms": round(ms, 4), "launches_per_step": n / nb},
        "kernels": kern,
        "model_tflops_per_step": round(step_tf, 3), "model_tflops_per_s": round(step_tf * args.steps / dt, 2),
        "mfu": round(step_tf * args.steps / dt / PEAK_BF16_TFLOPS, 4), "final_loss": round(loss, 5),
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
