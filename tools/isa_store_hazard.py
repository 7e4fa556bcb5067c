"""Scans hipcc device assembly for the VMEM-store data hazard: a `*_store_dwordx3/x4` (or b96/b128) whose
data VGPRs are overwritten by the very next instruction (no wait state). The store reads its data registers
after issue; hipcc (ROCm 7.2, gfx950) was seen to emit such pairs without the `s_nop` the hazard needs,
and the stored dwords then come out corrupted (SwiGLU backward epilogue, round 2). Exit status 1 if any.

  python tools/isa_store_hazard.py file.s [...]      (hipcc --cuda-device-only -S output)
"""
import re
import sys

STORE = re.compile(r"^\s*(buffer_store_dwordx[34]|global_store_dwordx[34]|flat_store_dwordx[34]|scratch_store_dwordx[34])\s+(?:(?:off|v\[\d+:\d+\]|v\d+),\s*)?v\[(\d+):(\d+)\]")
DEF = re.compile(r"^\s*(v_\w+|buffer_load\w*|global_load\w*|ds_read\w*|flat_load\w*)\s+v(?:\[(\d+):(\d+)\]|(\d+))")


def regs_def(line):
    m = DEF.match(line)
    if not m or m.group(1).startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    if m.group(4) is not None:
        return {int(m.group(4))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def scan(path):
    hits = []
    fn = "?"
    lines = open(path).read().splitlines()
    for i, ln in enumerate(lines):
        mf = re.match(r"^(_Z\w+):", ln)
        if mf:
            fn = mf.group(1)
        m = None
        # data operand of a store: global_store_dwordx4 vADDR, v[a:b], off  /  buffer_store_dwordx4 v[a:b], ...
        if "store_dwordx4" in ln or "store_dwordx3" in ln:
            toks = re.findall(r"v\[(\d+):(\d+)\]", ln)
            if ln.strip().startswith(("global_store", "flat_store", "scratch_store")) and len(toks) >= 1:
                a, b = toks[-1]
            elif toks:
                a, b = toks[0]
            else:
                continue
            data = set(range(int(a), int(b) + 1))
            j = i + 1
            while j < len(lines) and (not lines[j].strip() or lines[j].strip().startswith(";")):
                j += 1
            if j < len(lines) and regs_def(lines[j]) & data:
                hits.append((fn, i + 1, ln.strip(), lines[j].strip()))
    return hits


def main():
    bad = 0
    for p in sys.argv[1:]:
        for fn, ln, st, nxt in scan(p):
            bad += 1
            print(f"{p}:{ln}: {fn}\n    {st}\n    {nxt}")
    print(f"{bad} store-data hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
