"""Run one forward GEMM shape at one forced geometry a few times (a target for rocprofv3 counter passes).

  python tools/gemm_one.py M N K GEO [ITERS]
"""
import os
os.environ.setdefault("VPT_DIAG", "1")  # A/B switches live in libvpt_hip_diag.so only

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402

from vpt import ops  # noqa: E402


def main():
    M, N, K, geo = (int(a) for a in sys.argv[1:5])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    ops.lib.vpt_gemm_set_geometry(geo)
    for _ in range(iters):
        ops.linear(x, w, out=y)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
