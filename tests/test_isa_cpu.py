"""Static check of the generated gfx950 device code (CPU only: hipcc cross-compiles): no 16-B / 12-B vector
store whose data registers the very next instruction overwrites (tools/isa_store_hazard.py). hipcc (ROCm 7.2)
was seen to emit exactly that in the fused SwiGLU-backward epilogue, which then stored corrupted dwords."""

import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "vision-pt_amd"))
sys.path.insert(0, str(ROOT / "tools"))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_no_vector_store_data_hazards(tmp_path):
    from vpt import _build
    import isa_store_hazard as H

    bad = []
    for src in sorted(_build.CSRC.glob("*.hip")):
        out = tmp_path / (src.stem + ".s")
        cmd = [_build.HIPCC, *[f for f in _build.CFLAGS if f != "-fPIC"], *_build.UNIT_FLAGS.get(src.name, []),
               "--cuda-device-only", "-S", str(src), "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        bad += H.scan(str(out))
    assert not bad, "\n".join(f"{fn} line {ln}: {st} -> {nxt}" for fn, ln, st, nxt in bad[:10])
