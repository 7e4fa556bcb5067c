"""The data-parallel path over RCCL itself (torch.distributed backend "nccl" = RCCL on ROCm) on the one GPU of the test
box: a process group of size 1 initialised exactly as bench.py does at N > 1 (`init_process_group("nccl",
device_id=...)` before any other GPU call), and GradSync / LossLog with force_collective=True, so every bucket's
bf16 wire cast and all-reduce, RCCL's stream-ordered `work.wait()` inside the side-stream context (overlap) and the
LossLog pinned-copy path run under RCCL's semantics rather than gloo's blocking ones.

Asserted (reference: src/trainer/common.py:219, 376-388; src/models/for_training.py:98-109, 171-183):
  - the backend is nccl;
  - overlap=True (each bucket stepped on a side stream behind its RCCL reduction) == the serial per-bucket path,
    bitwise, for parameters and the f32 optimizer state, with no clipping, clip-by-norm and clip-by-value;
  - the reduced wire gradient == the bf16 rounding of the rank's own f32 gradient (a SUM over one rank);
  - the clip coefficient formed on the device == torch's clip_grad_norm_ on that gradient;
  - LossLog returns the pushed losses exactly, in order.
The 8-GPU run (BASELINE config 4) is the driver's; RCCL refuses two ranks on one GPU."""
import io
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
LR = 1e-2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)  # as bench.py, before any GPU work
    from tests.test_ddp_gpu import _batch, _opt, _step, _trainer
    from vpt.ddp import GradSync, LossLog, grad_buckets
    res = {"backend": dist.get_backend()}
    b = _batch(dev)
    sl = slice(0, 4)
    # the reduced gradient of one step, and clip thresholds that bind
    tr, cfg = _trainer(dev)
    sync = GradSync(tr.engine.grads, grad_buckets(tr.engine.layout, cfg.depth), wire="bf16", overlap=False,
                    force_collective=True)
    _step(tr, b, sl, dev, on_ready=sync.launch)
    sync.launch_rest()
    red = torch.zeros_like(tr.engine.grads)
    sync.finish(lambda lo, hi, sc, g: red[lo:hi].copy_(g.float() * sc))
    torch.cuda.synchronize()
    res["wire_equal"] = torch.equal(red, tr.engine.grads.bfloat16().float())
    max_norm = 0.5 * red.norm().item()
    max_value = 0.25 * red.abs().max().item()
    res["max_norm"], res["red"] = max_norm, red.cpu()
    for mode in ("none", "norm", "value"):
        kw = dict(clip_grad_norm=max_norm if mode == "norm" else None,
                  clip_grad_value=max_value if mode == "value" else None)
        out = {}
        for path in ("overlap", "serial"):
            tr, cfg = _trainer(dev)
            opt = _opt(tr)
            sync = GradSync(tr.engine.grads, grad_buckets(tr.engine.layout, cfg.depth), wire="bf16",
                            overlap=path == "overlap", force_collective=True, **kw)
            coef = []
            for k in range(2):
                s = opt.begin_step()
                fn = lambda lo, hi, sc, g, **kw2: opt.apply_range(s, lo, hi, sc, g, **kw2)  # noqa: E731
                if path == "overlap":
                    sync.arm(fn)
                _step(tr, b, sl, dev, on_ready=sync.launch)
                sync.launch_rest()
                if path == "overlap":
                    sync.finish()
                else:
                    sync.finish(fn)
                opt.end_step(s)
                if k == 0 and sync.clip_norm is not None:
                    torch.cuda.synchronize()
                    coef.append((sync.coef.item(), sync.norm.item()))
            torch.cuda.synchronize()
            out[path] = dict(y=tr.engine.params.cpu(), z=opt.z.cpu(), side=sync.side is not None, coef=coef,
                             moved=not torch.equal(opt.z, tr.engine.params.float()))
        res[mode] = out
    log = LossLog(dev, force_collective=True)
    vals = [0.25, 1.5, 3.0, 0.125]
    got = [log.push(torch.tensor(v, device=dev)) for v in vals]
    got = [x for x in got if x is not None]
    while log.pending:
        got.append(log.pop())
    res["losses"] = got
    res["loss_collective"] = log.collective
    buf = io.BytesIO()
    torch.save(res, buf)
    q.put(buf.getvalue())
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_world1_forced_collective_exact_path():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    r = torch.load(io.BytesIO(q.get(timeout=300)), weights_only=True)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert r["backend"] == "nccl"
    assert r["wire_equal"]
    for mode in ("none", "norm", "value"):
        o, s = r[mode]["overlap"], r[mode]["serial"]
        assert o["side"] and not s["side"]
        assert o["moved"]
        for k in ("y", "z"):
            assert torch.equal(o[k], s[k]), (mode, k)
    assert not torch.equal(r["value"]["overlap"]["z"], r["none"]["overlap"]["z"])  # the clamp binds
    (coef, norm), = r["norm"]["overlap"]["coef"]
    assert r["norm"]["serial"]["coef"][0][0] == coef
    g = r["red"].double()
    pp = torch.nn.Parameter(torch.zeros_like(g))
    pp.grad = g.clone()
    total = torch.nn.utils.clip_grad_norm_([pp], r["max_norm"]).item()
    assert abs(norm - total) <= 1e-6 * total, (norm, total)
    assert abs(coef - min(1.0, r["max_norm"] / (total + 1e-6))) <= 1e-6 and coef < 1.0
    assert r["loss_collective"]
    assert r["losses"] == [0.25, 1.5, 3.0, 0.125]
