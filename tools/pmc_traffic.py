"""Per-launch HBM traffic of the bench's probed ops from two rocprofv3 counter passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950: MI355X_MICROARCH.md §rocprofv3 PMC slots).

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KTRACE_DIR OUT.json [MFMA_DIR] [--tag TAG]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming read (16 B per lane,
global_load and LDS-DMA alike) -- every operand load of the GEMM and attention kernels is such a
read -- so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B streaming stores.
The kernel-trace stats of the same command give each op's mean duration per launch (sum of its
kernels' durations / launches), to check against bench.py's HIP-event probe.
"""

import collections
import csv
import glob
import json
import sys

# op -> (kernel-name substrings that belong to it, the substring counted as one launch of the op)
# A kernel counts toward every op whose members it matches (the R2 ring, gemm_r2.hip, is both a GEMM-family launch and,
# in the JiT step, only the fused SwiGLU-backward dgrad: its own entry; in the config-5 step it is the 128x128 LoRA
# GEMMs of geometry 1281, the same kernel name, reported as gemm_r2).
OPS = {
    "gemm": (("gemm_ring_kernel", "gemm_bf16_kernel", "gemm_r2_kernel", "splitk_reduce_kernel"),
             ("gemm_ring_kernel", "gemm_bf16_kernel", "gemm_r2_kernel")),
    "swb_dgrad_r2": (("gemm_r2_kernel",), ("gemm_r2_kernel",)),
    "attn_fwd": (("attn_fwd_kernel",), ("attn_fwd_kernel",)),
    "attn_bwd": (("attn_bwd_pre_kernel", "attn_bwd_kernel", "attn_bwd_dkdv_kernel", "attn_bwd_dq_kernel"),
                 ("attn_bwd_kernel", "attn_bwd_dkdv_kernel")),
    # the GEMM family by kernel geometry: the 128 x 128 tile kernel and the 256 x 256 ring (each with its split-K
    # reduces counted in the family entry above only)
    "gemm_t128": (("gemm_bf16_kernel",), ("gemm_bf16_kernel",)),
    "gemm_ring256": (("gemm_ring_kernel",), ("gemm_ring_kernel",)),
    "gemm_r2": (("gemm_r2_kernel",), ("gemm_r2_kernel",)),
}


def _ops_of(name):
    return [op for op, (members, _) in OPS.items() if any(m in name for m in members)]


def _counter(dirname, counter):
    path = glob.glob(f"{dirname}/**/*counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(float)
    launches = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for op in _ops_of(r["Kernel_Name"]):
            tot[op] += float(r["Counter_Value"])
            if any(m in r["Kernel_Name"] for m in OPS[op][1]):
                launches[op] += 1
    return tot, launches


def _counters(dirname, names):
    """{op: {counter: sum over the op's dispatches}}, dispatches per op (counted once per launch kernel)."""
    path = glob.glob(f"{dirname}/**/*counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] not in names:
            continue
        for op in _ops_of(r["Kernel_Name"]):
            tot[op][r["Counter_Name"]] += float(r["Counter_Value"])
            if any(m in r["Kernel_Name"] for m in OPS[op][1]):
                seen[op].add(r.get("Dispatch_Id", r.get("Correlation_Id", len(seen[op]))))
    return tot, {op: len(v) for op, v in seen.items()}


def main():
    args = sys.argv[1:]
    tag = None
    if "--tag" in args:
        i = args.index("--tag")
        tag = args[i + 1]
        del args[i:i + 2]
    c5 = "--c5" in args
    if c5:
        args.remove("--c5")
    fdir, wdir, kdir, out = args[:4]
    mdir = args[4] if len(args) > 4 else None
    fetch, nf = _counter(fdir, "FETCH_SIZE")
    write, nw = _counter(wdir, "WRITE_SIZE")
    stats = glob.glob(f"{kdir}/**/*kernel_stats.csv", recursive=True)[0]
    dur = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(stats)):
        for op in _ops_of(r["Name"]):
            dur[op] += float(r["TotalDurationNs"])
            if any(m in r["Name"] for m in OPS[op][1]):
                calls[op] += int(r["Calls"])
    res = {}
    for op in OPS:
        if not nf[op] or not nw[op]:
            continue
        rd = 2.0 * fetch[op] * 1024 / nf[op]
        wr = write[op] * 1024 / nw[op]
        res[op] = {
            "hbm_bytes_per_launch": round(rd + wr),
            "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
            "fetch_size_kib_per_launch_raw": round(fetch[op] / nf[op], 1),
            "launches_pmc": nf[op],
            "rocprof_mean_ms_per_launch": round(dur[op] / calls[op] / 1e6, 4) if calls[op] else None,
            "rocprof_launches": calls[op],
        }
    if tag:
        res["_tag"] = tag
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of the same "
                      "command; read bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count of 16-B/lane reads), "
                      "write bytes = WRITE_SIZE x 1024; per launch of the op")
    if mdir:
        # MFMA pipe utilisation: SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over SIMDs
        # (MI355X_MICROARCH.md: 32 x N for 32x32x16 bf16); GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
        # the kernel's cycles = GUI_ACTIVE / 8 and the chip's SIMD-cycles = that x 1024 SIMDs.
        names = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")
        tot, n = _counters(mdir, names)
        for op, c in tot.items():
            if op not in res or not n.get(op):
                continue
            gui = c.get("GRBM_GUI_ACTIVE", 0.0)
            busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            d = res[op]
            d["mfma_busy_cycles_per_launch"] = round(busy / n[op])
            d["gui_active_per_launch"] = round(gui / n[op])
            d["sq_busy_cycles_per_launch"] = round(c.get("SQ_BUSY_CYCLES", 0.0) / n[op])
            if gui:
                d["mfma_util"] = round(busy * 8 / (gui * 1024), 4)
        res["_mfma_method"] = ("rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (one pass); "
                               "mfma_util = MFMA_BUSY x 8 / (GRBM_GUI_ACTIVE x 1024 SIMDs)")
    if c5 and "gemm" in res:
        # the C5 step's GEMM kernels (gemm_ring / gemm_bf16 + split-K reduces) are its base+LoRA GEMMs (842 launches per
        # step in the bench's probe) and 68 plain ones (conditioning MLPs, skeleton maps): the kernel names do not tell
        # them apart, so the LoRA GEMM's entry is the per-launch mean over all of them (LoRA launches: ~93 % of the
        # launches, ~96 % of the GEMM time)
        res["gemm_lora"] = dict(res["gemm"], note="per-launch mean over every GEMM-kernel dispatch of the C5 step "
                                                  "(842 base+LoRA + 68 plain GEMM launches per step)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
