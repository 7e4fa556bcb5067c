"""Builds libvpt_hip.so (gfx950) from vision-pt_amd/csrc/*.hip with hipcc, in-tree.

Each translation unit is compiled in parallel to build/*.o and linked into lib/libvpt_hip.so.
A unit is rebuilt only when its source or common.h is newer than its object.
"""

from __future__ import annotations

import concurrent.futures as cf
import os
import re
import subprocess
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent  # vision-pt_amd/
CSRC = PKG_ROOT / "csrc"
BUILD = PKG_ROOT / "build"
LIB = PKG_ROOT / "lib" / "libvpt_hip.so"
# diagnostic twin (-DVPT_DIAG): process-wide A/B switches and timing ablations for tools/ only
BUILD_DIAG = PKG_ROOT / "build_diag"
LIB_DIAG = PKG_ROOT / "lib" / "libvpt_hip_diag.so"
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
# Per-unit extra flags. gemm.hip, attention.hip: no SLP packing of f32 math into v_pk_*_f32 (packed f32 ops beside
# MFMAs cost issue cycles: guide, 'price of one filler beside MFMAs'; attention backward -1.9 %, r05a in-process A/B).
UNIT_FLAGS = {"gemm.hip": ["-fno-slp-vectorize"], "gemm_r2.hip": ["-fno-slp-vectorize"],
              "attention.hip": ["-fno-slp-vectorize"]}


def _needs(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _headers(src: Path) -> list[Path]:
    """csrc/*.h files a source includes, directly or through another header."""
    out, todo = [], [src]
    while todo:
        for name in re.findall(r'#include "([^"/]+\.h)"', todo.pop().read_text()):
            h = CSRC / name
            if h.exists() and h not in out:
                out.append(h)
                todo.append(h)
    return sorted(out)


def _compile(src: Path, diag: bool = False, bdir: Path | None = None, flags: dict | None = None) -> Path:
    obj = (bdir or (BUILD_DIAG if diag else BUILD)) / (src.stem + ".o")
    unit_flags = UNIT_FLAGS if flags is None else flags
    text = src.read_text()
    # diag/*.inc: a dependency of the units that include it (directly or through another .inc)
    incs = [f for f in sorted((CSRC / "diag").glob("*.inc")) if f.name in text] if diag else []
    incs += [f for f in sorted((CSRC / "diag").glob("*.inc")) if diag and any(f.name in i.read_text() for i in incs)]
    deps = [src] + _headers(src) + incs
    if _needs(obj, deps):
        cmd = [HIPCC, *CFLAGS, *unit_flags.get(src.name, []), *(["-DVPT_DIAG"] if diag else []), "-c", str(src), "-o",
               str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-4000:]}")
    return obj


def _gen_diag_sources() -> None:
    """csrc/diag/ring4_agpr.inc (the 4-wave ring GEMM's fixed-AGPR accessors) from its generator."""
    gen, inc = CSRC / "diag" / "gen_ring4_agpr.py", CSRC / "diag" / "ring4_agpr.inc"
    if not inc.exists() or inc.stat().st_mtime < gen.stat().st_mtime:
        r = subprocess.run([sys.executable, str(gen)], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{gen.name} failed:\n{r.stderr[-2000:]}")


def build(verbose: bool = False, diag: bool = False) -> Path:
    """Production library (default) or its diagnostic twin (diag=True, -DVPT_DIAG)."""
    bdir, lib = (BUILD_DIAG, LIB_DIAG) if diag else (BUILD, LIB)
    if diag:
        _gen_diag_sources()
    bdir.mkdir(exist_ok=True)
    lib.parent.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    workers = min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(lambda s: _compile(s, diag), srcs))
    if _needs(lib, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(lib)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    if verbose:
        print(f"built {lib}")
    return lib


def build_variant(name: str, flags: dict, diag: bool = False) -> Path:
    """tools/ only: the same sources with other per-unit flags (e.g. {"attention.hip": ["-fno-slp-vectorize"]}), into
    build_var/<name>/ and lib/var/libvpt_hip_<name>.so, for an in-process A/B against the production library
    (vpt._lib.load_library / use_library). Rebuilt from scratch every call (the flags are not tracked)."""
    bdir = PKG_ROOT / "build_var" / name
    lib = PKG_ROOT / "lib" / "var" / f"libvpt_hip_{name}.so"
    if diag:
        _gen_diag_sources()
    bdir.mkdir(parents=True, exist_ok=True)
    lib.parent.mkdir(parents=True, exist_ok=True)
    for o in bdir.glob("*.o"):
        o.unlink()
    srcs = sorted(CSRC.glob("*.hip"))
    base_flags = UNIT_FLAGS

    def obj(src):  # a unit whose flags match the production (or diag) build links that build's object, rebuilt if stale
        if flags.get(src.name, []) == base_flags.get(src.name, []):
            return _compile(src, diag)
        return _compile(src, diag, bdir, flags)

    with cf.ThreadPoolExecutor(min(len(srcs), 8)) as ex:
        objs = list(ex.map(obj, srcs))
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(lib)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    return lib


if __name__ == "__main__":
    build(verbose=True, diag="--diag" in sys.argv)
