"""Which torch (non-HIP-extension) kernels does one C5 step launch, and from where: torch.profiler over one
SDXLFlowMatchQLoRA.step after warm-up, aten ops grouped by (op, innermost vpt/ frame). Prints JSON.

  python tools/c5_torch_ops.py
"""
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from vpt.sdxl_flow import SDXLFlowMatchQLoRA  # noqa: E402


def main():
    m = SDXLFlowMatchQLoRA(B=4, device="cuda", seed=0)
    lat, ctx, pooled, sizes = m.make_inputs(seed=1)
    for _ in range(2):
        m.step(lat, ctx, pooled, sizes)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        m.step(lat, ctx, pooled, sizes)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.name in ("aten::empty", "aten::empty_strided", "aten::view",
                                                              "aten::as_strided", "aten::slice", "aten::select",
                                                              "aten::t", "aten::transpose", "aten::reshape",
                                                              "aten::_reshape_alias", "aten::unsqueeze", "aten::lift_fresh",
                                                              "aten::alias", "aten::detach", "aten::expand", "aten::item",
                                                              "aten::_local_scalar_dense", "aten::result_type", "aten::resolve_conj",
                                                              "aten::resolve_neg", "aten::empty_like", "aten::is_nonzero"):
            continue
        frame = next((f for f in (ev.stack or []) if "/vpt/" in f), "?")
        cnt[(ev.name, frame.split("vision-pt_amd/")[-1])] += 1
    top = [{"op": k[0], "at": k[1], "calls": v} for k, v in cnt.most_common(40)]
    print(json.dumps({"total_aten_calls": sum(cnt.values()), "top": top}, indent=1))


if __name__ == "__main__":
    main()
