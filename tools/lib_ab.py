"""In-process A/B of builds of the same C ABI (compile-flag or code variants built by vpt._build.build_variant into
lib/var/libvpt_hip_<name>.so; "base" = the production lib/libvpt_hip.so): every library is loaded once, and calls are
routed through each in turn (vpt._lib.use_library), interleaved over rounds, so allocation, clocks and box are shared.

  attn : attention forward (fixed reference) and backward at the C3 shape (JiT-B/16, B=8, 1024^2: n = 4170 rows,
         4106 always-valid keys, 12 heads, QK-normed inputs), HIP events on the launching stream, per-launch medians;
         outputs compared bitwise with "base".
  step : the C3 training step (B=8, the 5 buckets round-robin, fused optimizer), ms per step medians.
  swb  : the SwiGLU-backward dgrad (dY . W3 with the SwiGLU backward in the epilogue) at the C3 shape (M = 33360,
         F = 2048, D = 768), per-launch medians; dx12 compared bitwise with the first variant.

  python tools/lib_ab.py --variants base,noslp [--what attn,step] [--rounds 6]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vpt import _lib, ops  # noqa: E402
from vpt._build import LIB, PKG_ROOT  # noqa: E402


def lib_path(name):
    return LIB if name == "base" else PKG_ROOT / "lib" / "var" / f"libvpt_hip_{name}.so"


def attn_case(dev):
    B, H, n, nd = 8, 12, 4170, 4106
    D = 64 * H
    M = B * n
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(M, 3 * D, device=dev, generator=g).bfloat16()
    wq = (1 + 0.1 * torch.randn(64, device=dev, generator=g)).bfloat16()
    wk = (1 + 0.1 * torch.randn(64, device=dev, generator=g)).bfloat16()
    ang = torch.rand(n, 32, device=dev, generator=g) * 6
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    qk = ops.qknorm_rope_fwd(qkv, wq, wk, cos, sin, n, q_scale=ops.attn_q_scale(0.125))
    kb = torch.zeros(B, n, device=dev)
    kb[:, nd + 30:] = float("-inf")
    o = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, n, device=dev)
    do = torch.randn(M, D, device=dev, generator=g).bfloat16()
    dqkv = torch.zeros(M, 3 * D, dtype=torch.bfloat16, device=dev)
    dqk = torch.zeros(M, 2 * D, dtype=torch.bfloat16, device=dev)
    delta = torch.empty(B, H, n, device=dev)
    q4, k4, v4 = ops._t4(qk, B, n, H, 0), ops._t4(qk, B, n, H, D), ops._t4(qkv, B, n, H, 2 * D)
    o4, do4 = ops._t4(o, B, n, H, 0), ops._t4(do, B, n, H, 0)

    def fwd():
        ops.attn_fwd_qknorm(q4, k4, v4, o4, lse, kb, wq, wk, B, H, n, n, nd)

    def bwd():
        ops.attn_bwd(q4, k4, v4, o4, do4, lse, delta, kb, ops._t4(dqk, B, n, H, 0), ops._t4(dqk, B, n, H, D),
                     ops._t4(dqkv, B, n, H, 2 * D), B, H, n, n, nd)

    def check(heads=2):
        """max |error| of o and of lse (log2 units, stored negated) vs a torch fp32 reference, batch 0, heads < `heads`."""
        eo, el = 0.0, 0.0
        for h in range(heads):
            q = qk[:n, h * 64:(h + 1) * 64].float()
            k = qk[:n, D + h * 64:D + (h + 1) * 64].float()
            v = qkv[:n, 2 * D + h * 64:2 * D + (h + 1) * 64].float()
            s = q @ k.T + kb[0][None, :]                     # log2 units (q pre-scaled by scale * log2 e)
            ref_lse = -torch.logsumexp(s * 0.6931471805599453, 1) / 0.6931471805599453
            ref_o = torch.softmax(s * 0.6931471805599453, 1) @ v
            el = max(el, (lse[0, h] - ref_lse).abs().max().item())
            eo = max(eo, (o[:n, h * 64:(h + 1) * 64].float() - ref_o).abs().max().item())
        return {"o_max_abs_err": eo, "lse_max_abs_err": el}

    return fwd, bwd, (o, lse, dqk, dqkv), check


def time_launches(fn, iters):
    st = torch.cuda.current_stream()
    fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    ev[0].record(st)
    for i in range(iters):
        fn()
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    return statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(iters))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base,noslp")
    ap.add_argument("--what", default="attn,step")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    names = args.variants.split(",")
    libs = {nm: _lib.load_library(lib_path(nm)) for nm in names}
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"variants": names}
    what = args.what.split(",")
    if "attn" in what:
        fwd, bwd, res, check = attn_case(dev)
        ref = None
        eq, err = {}, {}
        for rep in range(2):  # each variant twice, in turn: run-to-run and library-to-library equality
            for nm in names:
                _lib.use_library(libs[nm])
                fwd()
                torch.cuda.synchronize()
                if rep == 0:
                    err[nm] = check()
                bwd()
                torch.cuda.synchronize()
                got = [t.clone() for t in res]
                if ref is None:
                    ref = got
                eq[f"{nm}#{rep}"] = {k: (torch.equal(a, b), (a.float() - b.float()).abs().max().item())
                                     for k, a, b in zip(("o", "lse", "dqk", "dqkv"), ref, got)}
        tm = {f"{k}_{nm}": [] for k in ("fwd", "bwd") for nm in names}
        for r in range(args.rounds):
            order = names if r % 2 == 0 else names[::-1]
            for nm in order:
                _lib.use_library(libs[nm])
                tm[f"fwd_{nm}"].append(time_launches(fwd, args.iters))
                tm[f"bwd_{nm}"].append(time_launches(bwd, args.iters))
        med = {k: round(statistics.median(v), 4) for k, v in tm.items()}
        out["attn"] = {"bitwise_equal_to_first": eq, "fwd_vs_fp32": err, "median_ms": med,
                       "ratio_to_first": {k: round(v / med[k.split("_")[0] + "_" + names[0]], 4) for k, v in med.items()}}
        print(json.dumps(out["attn"]), flush=True)
    if "swb" in what:
        M, D, F = 8 * 4170, 768, 2048
        g = torch.Generator(device=dev).manual_seed(1)
        dy = torch.randn(M, D, device=dev, generator=g).bfloat16()
        w3 = (torch.randn(D, F, device=dev, generator=g) * 0.05).bfloat16()
        x12 = torch.randn(M, 2 * F, device=dev, generator=g).bfloat16()
        dx12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device=dev)
        ws = torch.empty(M, F, dtype=torch.bfloat16, device=dev)
        # a 512-MB sweep between launches evicts L2 / MALL as the step's other kernels do
        flush = torch.empty(128 << 20, dtype=torch.float32, device=dev)

        def swb():
            flush.zero_()
            ops.linear_dgrad_swiglu(dy, w3, x12, dx12, workspace=ws)

        ref, eq = None, {}
        for nm in names:
            _lib.use_library(libs[nm])
            swb()
            torch.cuda.synchronize()
            if ref is None:
                ref = dx12.clone()
            eq[nm] = torch.equal(ref, dx12)
        tm = {nm: [] for nm in names}
        for r in range(args.rounds):
            order = names if r % 2 == 0 else names[::-1]
            for nm in order:
                _lib.use_library(libs[nm])
                st = torch.cuda.current_stream()
                ts = []
                for _ in range(args.iters):
                    flush.zero_()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    ops.linear_dgrad_swiglu(dy, w3, x12, dx12, workspace=ws)
                    b.record(st)
                    ts.append((a, b))
                torch.cuda.synchronize()
                tm[nm].append(statistics.median(x.elapsed_time(y) for x, y in ts))
        med = {nm: round(statistics.median(v) * 1e3, 2) for nm, v in tm.items()}
        out["swb"] = {"bitwise_equal_to_first": eq, "median_us": med,
                      "ratio_to_first": {nm: round(v / med[names[0]], 4) for nm, v in med.items()}}
        print(json.dumps(out["swb"]), flush=True)
    if "step" in what:
        import bench
        from vpt.config import JiT_B_16_Config, JiTTrainingConfig
        from vpt.jit_train import JiTTrainer
        from vpt.optim import RAdamScheduleFreeFlat
        _lib.use_library(libs[names[0]])
        tr = JiTTrainer(JiT_B_16_Config(), bench.N_CLASSES, JiTTrainingConfig(loss_target="image"), device=dev, seed=1)
        tr.engine.init_weights(seed=0)
        opt = RAdamScheduleFreeFlat(tr.engine.params, tr.engine.grads, lr=1e-4)
        opt.train()
        batches = bench.make_batches(8, dev, seed=100)
        it = [0]

        def step():
            b = batches[it[0] % len(batches)]
            it[0] += 1
            tr.step(b["images"], b["ids"], b["mask"], b["original_size"], b["target_size"], b["crop_coords"])
            opt.step()

        for nm in names:
            _lib.use_library(libs[nm])
            for _ in range(len(batches)):
                step()
        torch.cuda.synchronize()
        tm = {nm: [] for nm in names}
        for r in range(args.rounds):
            order = names if r % 2 == 0 else names[::-1]
            for nm in order:
                _lib.use_library(libs[nm])
                step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    step()
                torch.cuda.synchronize()
                tm[nm].append((time.perf_counter() - t0) / args.steps * 1e3)
            print(f"round {r}: " + "  ".join(f"{nm} {tm[nm][-1]:.3f} ms" for nm in names), flush=True)
        med = {nm: statistics.median(v) for nm, v in tm.items()}
        out["step"] = {"median_ms": {k: round(v, 3) for k, v in med.items()},
                       "gain_vs_first": {k: round(med[names[0]] / v - 1, 4) for k, v in med.items()}}
        print(json.dumps(out["step"]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
