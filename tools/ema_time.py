"""EMA kernel timing: the 16-B path (aligned bases) vs the element-wise path (1-element offset), n = JiT-B/16's
parameter count order (131M bf16), HIP events on the launching stream, median of 20."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vision-pt_amd"))
import torch
from vpt import ops

n = 131_000_000
dev = torch.device("cuda:0")
e = torch.randn(n + 8, device=dev).bfloat16()
p = torch.randn(n + 8, device=dev).bfloat16()
out = {}
for name, off in (("vec16", 0), ("scalar", 1)):
    ts = []
    for _ in range(23):
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.ema_update(e[off:off + n], p[off:off + n], 0.9999, False)
        t.record()
        t.synchronize()
        ts.append(s.elapsed_time(t))
    ms = sorted(ts[3:])[10]
    out[name] = {"ms": round(ms, 4), "gb_s": round(n * 6 / ms / 1e6, 1)}
print(json.dumps(out))
