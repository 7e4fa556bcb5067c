"""bench.py under the diagnostic library with the ring GEMMs' grid forced (vpt_gemm_set_ring_grid): 256 = persistent
(one block per CU walking items), 0 = the default, one block per item -- for same-box A/B of the step with the side-stream
optimizer overlap on (--overlap on), where the optimizer's kernels share the chip with the backward's GEMMs.

  python tools/bench_ring_grid.py RING_GRID [bench.py args...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (before the library: HIP is initialised the way the bench does it)

from vpt import _lib  # noqa: E402

_lib.use_diag()

rg = int(sys.argv[1])
_lib.lib.vpt_gemm_set_ring_grid(rg)
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
