"""Builds libvpt_hip.so from csrc/ at another git revision into vision-pt_amd/lib/ab/<name>.so, for same-box
A/B timing (VPT_LIB_AB=<path> makes vpt load it instead of the production library).

  python tools/build_ab.py REV NAME [--diag]
"""
import importlib.util
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _build_module(rev: str, td: Path):
    """vpt/_build.py as of `rev` (its compiler flags, per-unit flags included)."""
    src = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:vision-pt_amd/vpt/_build.py"], capture_output=True,
                         check=True).stdout
    path = td / "_build_rev.py"
    path.write_bytes(src)
    spec = importlib.util.spec_from_file_location("_build_rev", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if not hasattr(mod, "UNIT_FLAGS"):
        mod.UNIT_FLAGS = {}
    return mod


def main():
    rev, name = sys.argv[1], sys.argv[2]
    diag = "--diag" in sys.argv
    out = ROOT / "vision-pt_amd" / "lib" / "ab" / f"{name}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        _build = _build_module(rev, td)
        # csrc/ and include/ at their repository paths (units include ../../include/vpt_hip.h)
        files = subprocess.run(["git", "-C", str(ROOT), "ls-tree", "--name-only", rev, "vision-pt_amd/csrc/",
                                "include/"], capture_output=True, text=True, check=True).stdout.split()
        for f in files:
            data = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:{f}"], capture_output=True, check=True).stdout
            (td / f).parent.mkdir(parents=True, exist_ok=True)
            (td / f).write_bytes(data)
        objs = []
        for src in sorted((td / "vision-pt_amd" / "csrc").glob("*.hip")):
            obj = td / (src.stem + ".o")
            cmd = [_build.HIPCC, *_build.CFLAGS, *_build.UNIT_FLAGS.get(src.name, []), *(["-DVPT_DIAG"] if diag else []),
                   "-c", str(src), "-o", str(obj)]
            subprocess.run(cmd, check=True)
            objs.append(str(obj))
        subprocess.run([_build.HIPCC, "-shared", "-fPIC", f"--offload-arch={_build.ARCH}", *objs, "-o", str(out)], check=True)
    print(out)


if __name__ == "__main__":
    main()
