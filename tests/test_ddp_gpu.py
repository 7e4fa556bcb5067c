"""The data-parallel path with the REAL HIP engine: two ranks on the one GPU of the test box (gloo carries
the CUDA tensors; the 8-GPU RCCL run is the driver's), each running JiTTrainer.step on its half of a batch
with GradSync.launch as the engine's on_ready hook (buckets reduced in backward-completion order, bf16 wire),
the rest launched after the class-embedding scatter, then the per-bucket finish. The averaged gradient must
equal a single-rank step on the whole batch (SURVEY §8(e) parity) and be identical on both ranks; every
bucket's reduction is applied exactly once."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _trainer(dev):
    from tests.golden import golden_configs as GC
    from vpt.config import DenoiserConfig, JiTTrainingConfig
    from vpt.jit_train import JiTTrainer
    oc = GC.micro_config()
    cfg = DenoiserConfig(hidden_size=oc.hidden_size, depth=oc.depth, num_heads=oc.num_heads,
                         bottleneck_dim=oc.bottleneck_dim, context_dim=oc.context_dim,
                         context_start_block=oc.context_start_block)
    tr = JiTTrainer(cfg, 20, JiTTrainingConfig(loss_target="image"), device=dev, seed=1)
    tr.engine.init_weights(seed=0)
    return tr, cfg


def _batch(dev):
    g = torch.Generator().manual_seed(7)
    B = 4
    img = (torch.rand(B, 3, 64, 48, generator=g) * 2 - 1).half()
    noise = torch.randn(B, 3, 64, 48, generator=g).half()
    t = torch.rand(B, generator=g) * 0.8 + 0.1
    ids = torch.randint(0, 20, (B, 8), generator=g)
    mask = torch.ones(B, 8, dtype=torch.long)
    mask[1, 5:] = 0
    mask[2, 3:] = 0
    ids = torch.where(mask.bool(), ids, torch.full_like(ids, 20))
    size = torch.tensor([[64, 48]] * B)
    return dict(img=img, noise=noise, t=t, ids=ids, mask=mask, size=size)


def _step(tr, b, sl, dev, on_ready=None):
    return tr.step(b["img"][sl].to(dev), b["ids"][sl], b["mask"][sl], b["size"][sl].to(dev), b["size"][sl].to(dev),
                   torch.zeros(b["size"][sl].shape, dtype=torch.long, device=dev), t=b["t"][sl],
                   noise=b["noise"][sl].to(dev), drop_context=False, on_ready=on_ready)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vpt.ddp import GradSync, grad_buckets
    tr, cfg = _trainer(dev)
    b = _batch(dev)
    sync = GradSync(tr.engine.grads, grad_buckets(tr.engine.layout, cfg.depth), wire="bf16")
    launched = []
    hook = lambda name: (launched.append(name), sync.launch(name))  # noqa: E731
    _step(tr, b, slice(rank * 2, rank * 2 + 2), dev, on_ready=hook)
    sync.launch_rest()
    out = torch.zeros_like(tr.engine.grads)
    applied = []
    sync.finish(lambda lo, hi, sc, g: (applied.append((lo, hi)), out[lo:hi].copy_(g.float() * sc)))
    torch.cuda.synchronize()
    q.put((rank, out.cpu(), launched, applied))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_real_engine_gradient_mean():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda t: t[0])
    g0, g1 = out[0][1], out[1][1]
    assert torch.equal(g0, g1)
    dev = torch.device("cuda", 0)
    tr, cfg = _trainer(dev)
    _step(tr, _batch(dev), slice(0, 4), dev)
    ref = tr.engine.grads.float().cpu()
    assert ((g0 - ref).norm() / ref.norm()).item() < 8e-3  # bf16 wire: rank grads and sum rounded to bf16
    # hook order = backward completion order: final layer first, then blocks last to first
    assert out[0][2] == ["final"] + [f"block{i}" for i in reversed(range(cfg.depth))]
    assert sum(hi - lo for lo, hi in out[0][3]) == tr.engine.layout.total
