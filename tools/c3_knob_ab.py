"""In-process A/B of the JiT engine's module-level switches (vpt.engine: FUSED_QKNORM_FWD, FUSED_QKNORM_BWD,
FIXREF_ATTN_FWD): one JiT-B/16 trainer at C3 (B=8, the 5 buckets round-robin, fused optimizer), then rounds of K timed
steps alternating the knob(s) on / off, so allocation, clocks and box are shared; medians of ms per step.

  python tools/c3_knob_ab.py FIXREF_ATTN_FWD [--rounds 6] [--steps 5]
  python tools/c3_knob_ab.py WGRAD_SPLIT_DIV=2/1      (a non-boolean engine attribute: NAME=ON/OFF)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from vpt import engine, ops  # noqa: E402
from vpt.config import JiT_B_16_Config, JiTTrainingConfig  # noqa: E402
from vpt.jit_train import JiTTrainer  # noqa: E402
from vpt.optim import RAdamScheduleFreeFlat  # noqa: E402


def _where(k):  # "NAME" = vpt.engine.NAME, "ops.NAME" = vpt.ops.NAME
    return (ops, k[4:]) if k.startswith("ops.") else (engine, k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knobs", help="comma-separated vpt.engine globals switched together (ops.NAME: a vpt.ops global)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--grad-ckpt", action="store_true", help="gradient checkpointing on")
    ap.add_argument("--workload", default="c3", choices=["c3", "c2"], help="c2: 512^2 buckets, B=16")
    args = ap.parse_args()
    knobs = args.knobs.split(",")
    # diagnostic-library switches (loads the diagnostic library): name -> setter(on)
    from vpt import _lib
    diag = {"ATTN_BWD_STAGES3": lambda on: _lib.lib.vpt_attn_set_bwd_stages(3 if on else 2),
            "SWB_AHEAD": lambda on: _lib.lib.vpt_gemm_set_swb_one_group(0 if on else 1),
            "ATTN_XCD": lambda on: _lib.lib.vpt_attn_set_xcd_order(1 if on else 0),
            "ATTN_FWD_ORD": lambda on: _lib.lib.vpt_attn_set_fwd_order(1 if on else 0),
            "ATTN_FWD_LSUM": lambda on: _lib.lib.vpt_attn_set_fwd_lsum(1 if on else 0),
            "ATTN_BWD_MF16": lambda on: _lib.lib.vpt_attn_set_bwd_mfma16(3 if on else 0),
            "ATTN_BWD_MF16_KV": lambda on: _lib.lib.vpt_attn_set_bwd_mfma16(1 if on else 0),
            "ATTN_BWD_MF16_Q": lambda on: _lib.lib.vpt_attn_set_bwd_mfma16(2 if on else 0),
            "ATTN_BWD_MF16_ORD": lambda on: _lib.lib.vpt_attn_set_bwd_mfma16(7 if on else 0),
            "ATTN_BWD_MF16_UNORD": lambda on: _lib.lib.vpt_attn_set_bwd_mfma16(3 if on else 7),
            "ATTN_FWD_MF16": lambda on: _lib.lib.vpt_attn_set_fwd_mfma16(1 if on else 0),
            "ATTN_DQ_ORD": lambda on: _lib.lib.vpt_attn_set_rows64(16 if on else 0),
            "ATTN_PF_KV": lambda on: _lib.lib.vpt_attn_set_bwd_prefetch(1 if on else 0),
            "ATTN_PF_Q": lambda on: _lib.lib.vpt_attn_set_bwd_prefetch(2 if on else 0),
            "ATTN_PF": lambda on: _lib.lib.vpt_attn_set_bwd_prefetch(3 if on else 0),
            "ATTN_DQ_ORD_NOPRIO": lambda on: _lib.lib.vpt_attn_set_bwd_prefetch(5 if on else 0),
            "ATTN_PRIO": lambda on: _lib.lib.vpt_attn_set_bwd_prefetch(4 if on else 0),
            "RING_PER_ITEM": lambda on: _lib.lib.vpt_gemm_set_ring_grid(0 if on else 256),
            # the 256x128 two-blocks-per-CU ring (gemm_r2.hip) by launch kind (vpt_gemm_set_r2 bit mask)
            "GEMM_R2": lambda on: _lib.lib.vpt_gemm_set_r2(31 if on else 8),
            "GEMM_R2_SWB": lambda on: _lib.lib.vpt_gemm_set_r2(8 if on else 0),
            "GEMM_R2_KMAJ": lambda on: _lib.lib.vpt_gemm_set_r2(9 if on else 8),
            "GEMM_R2_WGRAD": lambda on: _lib.lib.vpt_gemm_set_r2(10 if on else 8),
            "GEMM_R2_FWD": lambda on: _lib.lib.vpt_gemm_set_r2(28 if on else 8)}
    vals = {}  # NAME=ON/OFF: a non-boolean vpt.engine attribute and its two values
    for i, k in enumerate(knobs):
        if "=" in k:
            name, v = k.split("=")
            on, off = (int(x) for x in v.split("/"))
            knobs[i] = name
            vals[name] = (on, off)
    for k in knobs:
        if k in diag:
            if not _lib.DIAG:
                _lib.use_diag()
            continue
        if k not in vals and not isinstance(getattr(*_where(k)), bool):
            raise SystemExit(f"{k}: not a boolean knob of vpt.engine (NAME=ON/OFF for other values)")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = JiTTrainer(JiT_B_16_Config(), bench.N_CLASSES, JiTTrainingConfig(loss_target="image"), device=dev, seed=1)
    tr.engine.init_weights(seed=0)
    tr.engine.set_gradient_checkpointing(args.grad_ckpt)
    opt = RAdamScheduleFreeFlat(tr.engine.params, tr.engine.grads, lr=1e-4)
    opt.train()
    batches = (bench.make_batches(8, dev, seed=100) if args.workload == "c3"
               else bench.make_batches(16, dev, seed=100, buckets=bench.BUCKETS_C2))
    it = [0]

    def step():
        b = batches[it[0] % len(batches)]
        it[0] += 1
        tr.step(b["images"], b["ids"], b["mask"], b["original_size"], b["target_size"], b["crop_coords"])
        opt.step()

    def setk(v):
        for k in knobs:
            if k in diag:
                diag[k](v)
            elif k in vals:
                setattr(*_where(k), vals[k][0 if v else 1])
            else:
                setattr(*_where(k), v)

    for v in (True, False):
        setk(v)
        for _ in range(len(batches)):
            step()
    torch.cuda.synchronize()
    res = {"1": [], "0": []}
    for r in range(args.rounds):
        for v in ((True, False) if r % 2 == 0 else (False, True)):
            setk(v)
            step()  # one untimed step after the switch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            res["1" if v else "0"].append((time.perf_counter() - t0) / args.steps * 1e3)
        print(f"round {r}: on {res['1'][-1]:.3f} ms  off {res['0'][-1]:.3f} ms", flush=True)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(json.dumps({"knobs": knobs, "ms_per_step": {k: [round(x, 3) for x in v] for k, v in res.items()},
                      "median_ms": {k: round(v, 3) for k, v in med.items()},
                      "img_s_median": {k: round((8e3 if args.workload == "c3" else 16e3) / v, 3) for k, v in med.items()},
                      "gain": round(med["0"] / med["1"] - 1, 4)}))


if __name__ == "__main__":
    main()
