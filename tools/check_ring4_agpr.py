"""Check the 4-wave ring GEMM's register contract in a device assembly listing of gemm.hip (diag build):
its accumulators live in fixed AGPRs that only inline asm touches, so every gemm_ring4_kernel instance must
have no scratch (spills) and no compiler-generated instruction may name an AGPR.

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -DVPT_DIAG --cuda-device-only -S \\
      vision-pt_amd/csrc/gemm.hip -o /tmp/g.s && python tools/check_ring4_agpr.py /tmp/g.s
"""
import re
import sys


def check(path):
    s = open(path).read()
    ok = True
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
        name, desc = m.group(1), m.group(2)
        if "ring4" not in name:
            continue
        d = dict(re.findall(r"\.amdhsa_(\w+) (\S+)", desc))
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        body = s[i:j].split("\n")
        in_asm = False
        stray = []
        for line in body:
            if ";;#ASMSTART" in line:
                in_asm = True
            elif ";;#ASMEND" in line:
                in_asm = False
            elif not in_asm and re.search(r"\ba\d+\b|\ba\[\d+:\d+\]", line.split(";")[0]):
                stray.append(line.strip())
        scratch = int(d.get("private_segment_fixed_size", 0))
        good = scratch == 0 and not stray
        ok &= good
        print(f"{'ok  ' if good else 'FAIL'} {name[:80]} vgpr={d.get('next_free_vgpr')} "
              f"accum_offset={d.get('accum_offset')} scratch={scratch} stray_agpr={len(stray)} {stray[:3]}")
    return ok


if __name__ == "__main__":
    sys.exit(0 if check(sys.argv[1]) else 1)
