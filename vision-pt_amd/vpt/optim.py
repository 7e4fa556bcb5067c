"""RAdamScheduleFree as ONE fused HIP kernel over the flat parameter buffer.

Restates schedulefree==1.4.1 `RAdamScheduleFree` (the optimizer of configs/jit/x-loss/config.yml:74-78,
selected through src/optimizer/util.py:5-31; not installed in the reference's environment here, so
parity is unpinned — the update below follows the published algorithm):

  k = step count, beta2_t = beta2^(k+1), bc2 = 1 - beta2_t
  rho_inf = 2/(1-beta2) - 1, rho_t = rho_inf - 2 (k+1) beta2_t / bc2
  rect = sqrt((rho_t-4)(rho_t-2) rho_inf / ((rho_inf-4)(rho_inf-2) rho_t)) if rho_t > 4
         else (0 if silent_sgd_phase else 1)
  lr_t = lr * rect ; scheduled_lr = lr_t ; lr_max = max(lr_max, lr_t)
  weight = (k+1)^r * lr_max^weight_lr_power ; weight_sum += weight ; ckp1 = weight / weight_sum (0 if 0/0)
  v = beta2 v + (1-beta2) g^2 ; g <- g / (sqrt(v / bc2) + eps)  (only when rho_t > 4)
  g += wd * y ; y <- lerp(y, z, ckp1) ; y <- y + lr_t (beta1 (1-ckp1) - 1) g ; z <- z - lr_t g
  (y is the bf16 parameter: rounded after the lerp and after the add, as the reference's two
  in-place foreach ops on a bf16 tensor round it)
and train()/eval() swap y <-> x via p.lerp_(z, 1-beta1) / p.lerp_(z, 1-1/beta1).

Differences from the reference by design: z and v are kept in f32 (the reference keeps them in the
parameter dtype, bf16), gradients arrive in f32, and the optional `grad_scale` folds the DDP mean.
The param_groups dicts carry the same keys as schedulefree (incl. "scheduled_lr", which
src/trainer/common.py:499-514 reads).
"""

from __future__ import annotations

import math

import torch

from . import ops


class RAdamScheduleFreeFlat:
    def __init__(self, params: torch.Tensor, grads: torch.Tensor, lr: float = 0.0025, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, r: float = 0.0, weight_lr_power: float = 2.0,
                 silent_sgd_phase: bool = True):
        if params.dtype != torch.bfloat16 or grads.dtype != torch.float32 or params.numel() != grads.numel():
            raise ValueError("flat bf16 params and f32 grads of equal size expected")
        self.params, self.grads = params, grads
        self.z = torch.empty(params.numel(), dtype=torch.float32, device=params.device)
        self.v = torch.empty_like(self.z)
        self._initialised = False
        self.param_groups = [dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, r=r, k=0,
                                  train_mode=False, weight_sum=0.0, lr_max=-1.0, scheduled_lr=0.0,
                                  weight_lr_power=weight_lr_power, silent_sgd_phase=silent_sgd_phase)]

    @torch.no_grad()
    def train(self):
        g = self.param_groups[0]
        if not g["train_mode"]:
            if self._initialised:
                ops.sf_lerp(self.params, self.z, 1.0 - g["betas"][0])
            g["train_mode"] = True

    @torch.no_grad()
    def eval(self):
        g = self.param_groups[0]
        if g["train_mode"]:
            if self._initialised:
                ops.sf_lerp(self.params, self.z, 1.0 - 1.0 / g["betas"][0])
            g["train_mode"] = False

    def scalars(self) -> dict:
        """Host-side scalar schedule for the next step (pure arithmetic, no device work)."""
        g = self.param_groups[0]
        beta1, beta2 = g["betas"]
        step = g["k"] + 1
        beta2_t = beta2 ** step
        bc2 = 1 - beta2_t
        rho_inf = 2 / (1 - beta2) - 1
        rho_t = rho_inf - 2 * step * beta2_t / bc2
        if rho_t > 4.0:
            rect = math.sqrt((rho_t - 4.0) * (rho_t - 2.0) * rho_inf / ((rho_inf - 4.0) * (rho_inf - 2.0) * rho_t))
        else:
            rect = float(not g["silent_sgd_phase"])
        lr = g["lr"] * rect
        lr_max = max(lr, g["lr_max"])
        weight = (step ** g["r"]) * (lr_max ** g["weight_lr_power"])
        weight_sum = g["weight_sum"] + weight
        ckp1 = weight / weight_sum if weight_sum != 0 else 0.0
        return dict(step=step, bc2=bc2, adam=rho_t > 4.0, lr=lr, lr_max=lr_max, weight_sum=weight_sum, ckp1=ckp1,
                    adaptive_y_lr=lr * (beta1 * (1 - ckp1) - 1), beta2=beta2)

    @torch.no_grad()
    def begin_step(self) -> dict:
        """Computes this step's scalars; the update itself is applied range by range (so each
        all-reduced gradient bucket can be stepped as soon as it lands) and closed by end_step."""
        g = self.param_groups[0]
        if not g["train_mode"]:
            raise RuntimeError("Optimizer was not in train mode when step is called. "
                               "Please insert .train() and .eval() calls on the optimizer.")
        if not self._initialised:
            ops.sf_init(self.params, self.z, self.v)
            self._initialised = True
        return self.scalars()

    @torch.no_grad()
    def apply_range(self, s: dict, lo: int, hi: int, grad_scale: float = 1.0, grad: torch.Tensor | None = None,
                    clip_coef: torch.Tensor | None = None, clip_value: float | None = None):
        """Steps parameters [lo, hi) from self.grads[lo:hi], or from `grad` (f32 or bf16, the range's
        all-reduced wire buffer) when given. clip_coef (device f32 scalar) / clip_value: gradient clipping
        (for_training.py:98-109) applied to grad_scale * grad inside the same kernel."""
        g = self.param_groups[0]
        if hi <= lo:
            return
        src = self.grads[lo:hi] if grad is None else grad
        ops.radam_sf_step(self.params[lo:hi], src, self.z[lo:hi], self.v[lo:hi], beta2=s["beta2"],
                          bias_correction2=s["bc2"], eps=g["eps"], ckp1=s["ckp1"], adaptive_y_lr=s["adaptive_y_lr"],
                          lr=s["lr"], decay=g["weight_decay"], grad_scale=grad_scale, adam=s["adam"],
                          clip_coef=clip_coef, clip_value=clip_value or 0.0)

    def end_step(self, s: dict):
        g = self.param_groups[0]
        g["scheduled_lr"] = s["lr"]
        g["lr_max"] = s["lr_max"]
        g["weight_sum"] = s["weight_sum"]
        g["k"] = g["k"] + 1

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        s = self.begin_step()
        self.apply_range(s, 0, self.params.numel(), grad_scale)
        self.end_step(s)

    def zero_grad(self, set_to_none: bool = False):
        self.grads.zero_()

    def state_dict(self) -> dict:
        return {"param_groups": [dict(g) for g in self.param_groups], "z": self.z, "v": self.v,
                "initialised": self._initialised}
