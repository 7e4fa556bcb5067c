"""CPU, world_size 2 over gloo: the data-parallel gradient path (vpt.ddp) — bucket tiling of the
flat gradient buffer, per-bucket SUM all-reduce launched in backward order, mean folded into the
optimizer's grad_scale, and equivalence of an N-rank step to a 1-rank step at N x batch (the
SURVEY §8(e) parity definition), using the oracle model as the per-rank compute."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import jit_oracle as O
from tests.golden import golden_configs as GC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _vcfg(oc):
    from vpt.config import DenoiserConfig
    return DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                          bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                          context_start_block=oc.context_start_block)


def test_buckets_tile_flat_buffer():
    from vpt.config import JiT_B_16_Config
    from vpt.ddp import grad_buckets
    from vpt.params import ParamLayout
    for cfg, nc in ((JiT_B_16_Config(), 10000), (_vcfg(GC.micro_config()), 20)):
        lay = ParamLayout(cfg, nc)
        b = grad_buckets(lay, cfg.depth)
        spans = sorted((lo, hi) for _, lo, hi in b)
        assert spans[0][0] == 0 and spans[-1][1] == lay.total
        for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
            assert a1 == b0
        names = [n for n, _, _ in b]
        assert names[0] == "final" and names[1] == f"block{cfg.depth - 1}" and "embed" in names
        for s in lay.specs:  # every parameter lies inside exactly one bucket
            inside = [n for n, lo, hi in b if lo <= s.offset and s.offset + s.numel <= hi]
            assert len(inside) == 1, s.name


def _worker(rank, world, port, q, wire="f32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    from vpt.ddp import GradSync, LossLog, grad_buckets
    from vpt.params import ParamLayout
    oc = GC.micro_config()
    cfg = _vcfg(oc)
    lay = ParamLayout(cfg, 20)
    w = O.make_weights(oc, seed=1, n_classes=20)
    # each rank: its own half of a 4-image batch (rank-interleaved sampler semantics)
    full = GC.make_batch(oc, 4, 64, 48, 8, 20, seed=5, padded_rows=(1, 2))
    mine = {k: v[rank::world] for k, v in full.items()}
    model = O.load_weights(O.OracleJiT(oc), w)
    emb = w["class_encoder.embedding.weight"].clone().requires_grad_(True)
    loss, _ = O.train_step_loss(model, emb, mine, "image")
    loss.backward()
    grads = torch.zeros(lay.total)
    for n, p in model.named_parameters():
        s = lay.by_name[n]
        grads[s.offset:s.offset + s.numel] = p.grad.reshape(-1)
    s = lay.by_name["class_encoder.embedding.weight"]
    grads[s.offset:s.offset + s.numel] = emb.grad.reshape(-1)
    sync = GradSync(grads, grad_buckets(lay, cfg.depth), wire=wire)
    for name, _, _ in sync.buckets[:-2]:   # launched from the backward hook, in completion order
        sync.launch(name)
    sync.launch_rest()
    applied = []
    out = torch.zeros_like(grads)
    sync.finish(lambda lo, hi, sc, g: (applied.append((lo, hi)), out[lo:hi].copy_(g.float() * sc)))
    # per-step loss logging: accelerator.gather(loss).mean() as one 2-float all-reduce, read later
    log = LossLog("cpu", depth=2)
    first = log.push(loss.detach())
    second = log.push(loss.detach() * 3)
    third = log.pop()
    q.put((rank, out.clone(), applied, (first, second, third, loss.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["f32", "bf16"])
def test_two_rank_gradient_mean_equals_single_rank_big_batch(wire):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, wire)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda t: t[0])
    g0, g1 = out[0][1], out[1][1]
    assert torch.equal(g0, g1)  # every rank holds the same averaged gradient
    # reference: one process, whole batch of 4 (mean-of-means == mean because both halves have 2 images)
    from vpt.params import ParamLayout
    oc = GC.micro_config()
    lay = ParamLayout(_vcfg(oc), 20)
    w = O.make_weights(oc, seed=1, n_classes=20)
    full = GC.make_batch(oc, 4, 64, 48, 8, 20, seed=5, padded_rows=(1, 2))
    model = O.load_weights(O.OracleJiT(oc), w)
    emb = w["class_encoder.embedding.weight"].clone().requires_grad_(True)
    loss, _ = O.train_step_loss(model, emb, full, "image")
    loss.backward()
    ref = torch.zeros(lay.total)
    for n, p in model.named_parameters():
        s = lay.by_name[n]
        ref[s.offset:s.offset + s.numel] = p.grad.reshape(-1)
    s = lay.by_name["class_encoder.embedding.weight"]
    ref[s.offset:s.offset + s.numel] = emb.grad.reshape(-1)
    # f32 wire: exact up to summation order; bf16 wire (the reference DDP's bf16 .grad reduction):
    # two bf16 roundings of each rank's gradient and of the sum
    assert ((g0 - ref).norm() / ref.norm()).item() < (1e-5 if wire == "f32" else 8e-3)
    applied = out[0][2]
    assert sum(hi - lo for lo, hi in applied) == lay.total
    # loss log: mean over ranks of each pushed loss, returned one push later (depth 2)
    l0, l1 = out[0][3][3], out[1][3][3]
    for r in range(world):
        first, second, third, _ = out[r][3]
        assert first is None
        assert abs(second - (l0 + l1) / 2) < 1e-6 * abs(l0 + l1)
        assert abs(third - 3 * (l0 + l1) / 2) < 1e-6 * abs(l0 + l1)
