"""Debug: fused SwiGLU backward epilogue vs dgrad + elementwise kernel (mismatch statistics)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vision-pt_amd"))
import torch
from vpt import ops

def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).bfloat16().cuda()

M, D, F = 5192, 768, 2048
x = rnd(M, D, seed=130); w12 = rnd(2 * F, D, scale=0.03, seed=131); b12 = rnd(2 * F, scale=0.1, seed=132)
x12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device="cuda"); h = torch.empty(M, F, dtype=torch.bfloat16, device="cuda")
ops.linear_swiglu(x, w12, b12, x12, h)
dy = rnd(M, D, seed=133); w3 = rnd(D, F, scale=0.03, seed=134)
dx12 = torch.empty(M, 2 * F, dtype=torch.bfloat16, device="cuda")
ops.linear_dgrad_swiglu(dy, w3, x12, dx12)
dh = ops.linear_dgrad(dy, w3)
dx12_u = torch.empty_like(dx12)
ops.swiglu_bwd(dh, x12, dx12_u)
torch.cuda.synchronize()
for name, a, b in (("dx1", dx12[:, :F], dx12_u[:, :F]), ("dx2", dx12[:, F:], dx12_u[:, F:])):
    ne = (a != b)
    print(name, "mismatches", int(ne.sum()), "of", a.numel(), "max abs diff", (a.float() - b.float()).abs().max().item())
    idx = ne.nonzero()[:8].tolist()
    for r, c in idx:
        print("   ", r, c, a[r, c].item(), b[r, c].item(), "x1", x12[r, c].item(), "x2", x12[r, F + c].item(), "dh", dh[r, c].item())
    if ne.any():
        rows = ne.any(1).nonzero().flatten()
        cols = ne.any(0).nonzero().flatten()
        print("   rows", rows.min().item(), rows.max().item(), len(rows), "cols", cols.min().item(), cols.max().item(), len(cols))
