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
    q.put((rank, out.numpy().copy(), applied, (first, second, third, loss.item())))
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
    g0, g1 = torch.from_numpy(out[0][1]), torch.from_numpy(out[1][1])
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


# ----------------------------------------------------------------------- overlap, clipping, sharded order
def _grad_worker(rank, world, port, q, mode):
    """Each rank holds its own flat gradient over the micro layout; GradSync reduces the mean, lands every
    bucket as it is launched (overlap) or at finish (serial), with optional global-norm / value clipping; the
    callback applies the clip exactly as the optimizer kernel does (g * scale * coef, then clamp)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vpt.ddp import GradSync, grad_buckets
    from vpt.params import ParamLayout
    cfg = _vcfg(GC.micro_config())
    lay = ParamLayout(cfg, 20)
    g = torch.Generator().manual_seed(100 + rank)
    grads = torch.randn(lay.total, generator=g) * (1.0 + rank)
    mine = grads.clone()  # the all-reduce sums in place
    overlap, norm, value, accum = mode
    sync = GradSync(grads, grad_buckets(lay, cfg.depth), overlap=overlap, clip_grad_norm=norm, clip_grad_value=value)
    out = torch.full_like(grads, float("nan"))
    order = []

    def apply(lo, hi, sc, gr, clip_coef=None, clip_value=None):
        order.append((lo, hi))
        e = gr.float() * sc
        if clip_coef is not None:
            e = e * clip_coef
        if clip_value:
            e = e.clamp(-clip_value, clip_value)
        out[lo:hi] = e

    sync.arm(apply, 1.0 / accum)
    landed_during_backward = []
    for name, _, _ in sync.buckets[:-2]:  # the engine's on_ready calls, in completion order
        sync.launch(name)
        landed_during_backward.append(len(order))
    sync.launch_rest()
    sync.finish()
    q.put((rank, mine.numpy(), out.numpy(), order, landed_during_backward,
           sync.norm.item() if norm is not None else None))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *args)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize("mode", [(True, None, None, 1), (False, None, None, 1), (True, 1.0, None, 2),
                                  (False, 1.0, None, 1), (True, None, 0.05, 1), (True, 0.5, 0.02, 2)],
                         ids=["overlap", "serial", "overlap-clipnorm-accum2", "serial-clipnorm", "overlap-clipvalue",
                              "overlap-clipnorm-clipvalue-accum2"])
def test_two_rank_overlap_and_clipping_match_reference_semantics(mode):
    """World 2 over gloo: the mean gradient (SUM all-reduce x 1/world x 1/accum) with after_backward's
    clip_grad_norm_ then clip_grad_value_ (src/models/for_training.py:98-109) equals torch's own clipping of
    the mean gradient; with overlap every bucket is stepped as it is launched (none left for finish() except
    the two launched after the backward), unless global-norm clipping needs every bucket first."""
    overlap, norm, value, accum = mode
    res = [(r[0], torch.from_numpy(r[1]), torch.from_numpy(r[2]), *r[3:]) for r in _spawn(_grad_worker, 2, mode)]
    g_mean = (res[0][1] + res[1][1]) / 2 / accum
    ref = g_mean.clone()
    p = torch.nn.Parameter(torch.zeros_like(ref))
    p.grad = ref
    if norm is not None:
        tn = torch.nn.utils.clip_grad_norm_([p], norm)
        assert abs(res[0][5] - tn.item()) <= 1e-4 * tn.item()  # f32 sums in another order
    if value is not None:
        torch.nn.utils.clip_grad_value_([p], value)
    for r in range(2):
        out, order, landed = res[r][2], res[r][3], res[r][4]
        assert torch.allclose(out, p.grad, rtol=1e-5, atol=1e-7), (r, (out - p.grad).abs().max())
        spans = sorted(order)
        assert spans[0][0] == 0 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))  # each bucket once
        if overlap and norm is None:
            assert landed == list(range(1, len(landed) + 1))  # stepped during the backward, bucket by bucket
        else:
            assert all(n == 0 for n in landed)  # nothing stepped before finish()
    assert torch.equal(res[0][2], res[1][2])


def test_bench_shared_order_is_rank_interleaved():
    """bench.py's bucket schedule = accelerate prepare_data_loader over one shared seeded shuffle: the ranks'
    per-step draws interleave one permutation per epoch (so ranks hold different buckets in the same step), and
    world 1 is the plain per-epoch shuffle (every bucket once per epoch)."""
    import bench
    steps, nb = 20, 5
    for world in (1, 2, 4):
        per = [bench.shared_order(nb, steps, world, r) for r in range(world)]
        for e in range(steps // nb):
            merged = [per[j % world][e * nb + j // world] for j in range(nb * world)]
            assert sorted(merged) == sorted(i % nb for i in range(nb * world))  # one epoch = the shuffled list
        if world == 1:
            assert all(per[0].count(b) == steps // nb for b in range(nb))
    two = [bench.shared_order(nb, steps, 2, r) for r in range(2)]
    assert any(a != b for a, b in zip(*two))  # different buckets on the two ranks in some step


def _save_worker(rank, world, port, q, tmp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import types
    from vpt.trainer import JiTTrainLoop, SafetensorsSaver
    from vpt.params import ParamLayout
    cfg = _vcfg(GC.micro_config())
    lay = ParamLayout(cfg, 20)
    eng = types.SimpleNamespace(layout=lay, params=torch.full((lay.total,), float(rank)))
    loop = JiTTrainLoop.__new__(JiTTrainLoop)  # only the save path (no engine / optimizer needed)
    loop.trainer = types.SimpleNamespace(engine=eng)
    loop.savers = [SafetensorsSaver("jit", tmp)]
    loop.ema_savers, loop.ema, loop.saved = [], None, []
    loop._save(1, 4)
    q.put((rank, list(loop.saved)))
    dist.barrier()
    dist.destroy_process_group()


def test_checkpoint_saved_by_rank0_only(tmp_path):
    """common.py:390-423: wait_for_everyone, save on the main process only, wait_for_everyone."""
    from safetensors.torch import load_file
    res = _spawn(_save_worker, 2, str(tmp_path))
    assert len(res[0][1]) == 1 and res[1][1] == []
    files = sorted(os.listdir(tmp_path))
    assert files == ["jit_00001e_000004s.safetensors"]
    sd = load_file(os.path.join(tmp_path, files[0]))
    assert all(float(v.float().abs().max()) == 0.0 for v in sd.values())  # rank 0's replica


def test_integration_md_optimizer_callback_matches_gradsync():
    """The INTEGRATION.md §3 snippet's callback is called by GradSync with the arguments it passes (the round-2
    example had a 3-parameter lambda for a 4-argument call)."""
    import re
    import types
    from vpt.ddp import GradSync, grad_buckets
    from vpt.params import ParamLayout
    text = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), "INTEGRATION.md")).read()
    lam = re.search(r"sync\.arm\((lambda [^\n]*\))\)\n", text).group(1)
    calls = []
    opt = types.SimpleNamespace(apply_range=lambda s, lo, hi, sc, g, **kw: calls.append((lo, hi, sc, kw)))
    fn = eval(lam, {"opt": opt, "s": {}})
    cfg = _vcfg(GC.micro_config())
    lay = ParamLayout(cfg, 20)
    for clip in ({}, {"clip_grad_norm": 1.0, "clip_grad_value": 0.5}):
        calls.clear()
        sync = GradSync(torch.randn(lay.total), grad_buckets(lay, cfg.depth), **clip)
        sync.arm(fn)
        for n, _, _ in sync.buckets:
            sync.launch(n)
        sync.finish()
        assert sum(hi - lo for lo, hi, _, _ in calls) == lay.total
        assert all(set(kw) == ({"clip_coef", "clip_value"} if clip else set()) for *_, kw in calls)
