"""CPU restatement of schedulefree 1.4.1 `RAdamScheduleFree` (test infrastructure only).

The optimizer of the reference's JiT config (`/root/reference/configs/jit/x-loss/config.yml:74-78`,
built through `src/optimizer/util.py:5-31`; train()/eval() driven by `src/trainer/common.py:276-285`,
`scheduled_lr` read at `common.py:499-514`). schedulefree is not installed in this image, so this is a
restatement of the package's published step, NOT a run of it: RAdamScheduleFree parity is unpinned.

State z / exp_avg_sq is kept in f32 here, as the build keeps it (the package keeps it in the parameter
dtype); y (the parameter) is rounded to its dtype after each in-place op, as the package's foreach ops
round a bf16 parameter. Written independently of `vpt/optim.py` (it is the checker for it): per parameter tensor, in the
order of the package's foreach branch,

    exp_avg_sq = beta2 * exp_avg_sq + (1 - beta2) * g * g
    if rho_t > 4:  g = g / (sqrt(exp_avg_sq / bias_correction2) + eps)
    if decay:      g = g + decay * y
    y = lerp(y, z, ckp1);  y = y + adaptive_y_lr * g;  z = z - lr * g

with lr = group_lr * rect(rho_t) (0 in the silent-SGD warm-up), lr_max = max(lr_max, lr),
weight = step**r * lr_max**weight_lr_power, ckp1 = weight / weight_sum (0 when weight_sum == 0),
adaptive_y_lr = lr * (beta1 * (1 - ckp1) - 1); eval() sets y <- lerp(y, z, 1 - 1/beta1) and train()
y <- lerp(y, z, 1 - beta1).
"""

from __future__ import annotations

import math

import torch


class SFRef:
    def __init__(self, params: list[torch.Tensor], lr=0.0025, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, r=0.0,
                 weight_lr_power=2.0, silent_sgd_phase=True):
        self.params = params
        self.group = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, r=r, k=0, train_mode=False,
                          weight_sum=0.0, lr_max=-1.0, scheduled_lr=0.0, weight_lr_power=weight_lr_power,
                          silent_sgd_phase=silent_sgd_phase)
        self.z: list[torch.Tensor | None] = [None] * len(params)
        self.v: list[torch.Tensor | None] = [None] * len(params)

    @torch.no_grad()
    def train(self):
        g = self.group
        if not g["train_mode"]:
            for p, z in zip(self.params, self.z):
                if z is not None:
                    p.copy_(p.float().lerp(z, 1 - g["betas"][0]).to(p.dtype))
            g["train_mode"] = True

    @torch.no_grad()
    def eval(self):
        g = self.group
        if g["train_mode"]:
            for p, z in zip(self.params, self.z):
                if z is not None:
                    p.copy_(p.float().lerp(z, 1 - 1 / g["betas"][0]).to(p.dtype))
            g["train_mode"] = False

    @staticmethod
    def schedule(group: dict) -> dict:
        beta1, beta2 = group["betas"]
        step = group["k"] + 1
        beta2_t = beta2 ** step
        bc2 = 1 - beta2_t
        rho_inf = 2 / (1 - beta2) - 1
        rho_t = rho_inf - 2 * step * beta2_t / bc2
        if rho_t > 4.0:
            rect = ((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t)) ** 0.5
        else:
            rect = float(not group["silent_sgd_phase"])
        lr = group["lr"] * rect
        lr_max = max(lr, group["lr_max"])
        weight = (step ** group["r"]) * (lr_max ** group["weight_lr_power"])
        weight_sum = group["weight_sum"] + weight
        try:
            ckp1 = weight / weight_sum
        except ZeroDivisionError:
            ckp1 = 0.0
        return dict(bc2=bc2, rho_t=rho_t, lr=lr, lr_max=lr_max, weight_sum=weight_sum, ckp1=ckp1,
                    adaptive_y_lr=lr * (beta1 * (1 - ckp1) - 1))

    @torch.no_grad()
    def step(self, grads: list[torch.Tensor]):
        g = self.group
        if not g["train_mode"]:
            raise RuntimeError("not in train mode")
        s = self.schedule(g)
        g["scheduled_lr"], g["lr_max"], g["weight_sum"] = s["lr"], s["lr_max"], s["weight_sum"]
        beta2 = g["betas"][1]
        for i, (y, gr) in enumerate(zip(self.params, grads)):
            if self.z[i] is None:
                self.z[i] = y.detach().float().clone()
                self.v[i] = torch.zeros_like(self.z[i])
            z, v = self.z[i], self.v[i]
            gr = gr.float().clone()
            v.mul_(beta2).addcmul_(gr, gr, value=1 - beta2)
            if s["rho_t"] > 4.0:
                gr.div_(v.div(s["bc2"]).sqrt_().add_(g["eps"]))
            if g["weight_decay"] != 0:
                gr.add_(y.float(), alpha=g["weight_decay"])
            y.copy_(y.float().lerp(z, s["ckp1"]).to(y.dtype))
            y.copy_((y.float() + s["adaptive_y_lr"] * gr).to(y.dtype))
            z.sub_(gr, alpha=s["lr"])
        g["k"] += 1
        return s

    def x(self) -> list[torch.Tensor]:
        """The averaged iterate x (what eval() exposes) from y and z: y = (1-beta1) z + beta1 x."""
        b1 = self.group["betas"][0]
        return [y.float().lerp(z, 1 - 1 / b1) for y, z in zip(self.params, self.z)]


def reference_schedule(lr, betas, steps, r=0.0, weight_lr_power=2.0, silent_sgd_phase=True):
    """(scheduled lr, ckp1, adam?) for steps 1..steps."""
    grp = dict(lr=lr, betas=betas, r=r, k=0, weight_sum=0.0, lr_max=-1.0, weight_lr_power=weight_lr_power,
               silent_sgd_phase=silent_sgd_phase)
    out = []
    for _ in range(steps):
        s = SFRef.schedule(grp)
        grp["lr_max"], grp["weight_sum"], grp["k"] = s["lr_max"], s["weight_sum"], grp["k"] + 1
        out.append((s["lr"], s["ckp1"], s["rho_t"] > 4.0))
    return out

