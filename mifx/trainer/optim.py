"""TF-semantics optimizers for the PyTorch reference path.

The canned DNNLinearCombinedClassifier (`taxi_utils.py:186-191`) trains its DNN with Adagrad
(lr 0.05, initial accumulator 0.1) and its linear part with FTRL (lr = min(0.2, 1/sqrt(#cols)),
lr_power -0.5, initial accumulator 0.1). These match TF's ApplyAdagrad / ApplyFtrl update rules
exactly (no epsilon), as does the fused HIP optimizer in csrc/wide_deep.hip.
"""
from __future__ import annotations

import torch


class TFAdagrad(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 0.05, initial_accumulator_value: float = 0.1):
        super().__init__(params, dict(lr=lr, init=initial_accumulator_value))

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "acc" not in st:
                    st["acc"] = torch.full_like(p, g["init"])
                st["acc"].addcmul_(p.grad, p.grad)
                p.addcdiv_(p.grad, st["acc"].sqrt(), value=-g["lr"])


class Ftrl(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 0.2, lr_power: float = -0.5, initial_accumulator_value: float = 0.1,
                 l1: float = 0.0, l2: float = 0.0):
        super().__init__(params, dict(lr=lr, lr_power=lr_power, init=initial_accumulator_value, l1=l1, l2=l2))

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            lr, pw, l1, l2 = g["lr"], g["lr_power"], g["l1"], g["l2"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "acc" not in st:
                    st["acc"] = torch.full_like(p, g["init"])
                    st["lin"] = torch.zeros_like(p)
                acc, lin, grad = st["acc"], st["lin"], p.grad
                new_acc = acc + grad * grad
                if pw == -0.5:
                    sq_new, sq_old = new_acc.sqrt(), acc.sqrt()
                else:
                    sq_new, sq_old = new_acc.pow(-pw), acc.pow(-pw)
                lin.add_(grad - (sq_new - sq_old) / lr * p)
                quad = sq_new / lr + 2 * l2
                p.copy_(torch.where(lin.abs() > l1, (torch.sign(lin) * l1 - lin) / quad, torch.zeros_like(p)))
                acc.copy_(new_acc)


def make_optimizer(kind: str, params, lr: float, **kw) -> torch.optim.Optimizer:
    kind = kind.lower()
    if kind == "adagrad":
        return TFAdagrad(params, lr=lr, **kw)
    if kind == "ftrl":
        return Ftrl(params, lr=lr, **kw)
    if kind == "adam":
        return torch.optim.Adam(params, lr=lr, **kw)
    if kind == "sgd":
        return torch.optim.SGD(params, lr=lr, **kw)
    raise ValueError(f"unknown optimizer {kind}")


class FlatAdamW:
    """AdamW over a model whose parameters are re-homed as bf16 views of ONE flat buffer, with their
    gradients as views of one flat bf16 gradient buffer (autograd accumulates in place), and fp32
    master weights / moments kept here. `step()` is a single fused HIP launch (mifx.ops.adamw);
    `zero_grad()` is one memset. Both are hipGraph-capturable (device-side step counter)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 dtype: torch.dtype = torch.bfloat16):
        self.params = [p for p in params if p.requires_grad]
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.n = n
        self.flat = torch.empty(n, device=dev, dtype=dtype)
        self.flat_grad = torch.zeros(n, device=dev, dtype=dtype)
        self.master = torch.empty(n, device=dev, dtype=torch.float32)
        self.m = torch.zeros(n, device=dev, dtype=torch.float32)
        self.v = torch.zeros(n, device=dev, dtype=torch.float32)
        self.step_count = torch.zeros((), device=dev, dtype=torch.int32)
        off = 0
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                self.master[off:off + k].copy_(p.detach().reshape(-1).float())
                self.flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + k].view(p.shape)
                p.grad = self.flat_grad[off:off + k].view(p.shape)
                off += k

    def zero_grad(self, set_to_none: bool = False) -> None:  # grads stay views of the flat buffer
        self.flat_grad.zero_()

    def step(self) -> None:
        from ..ops.adamw import adamw_flat_

        adamw_flat_(self.flat, self.flat_grad, self.master, self.m, self.v, self.step_count, self.lr,
                    self.betas[0], self.betas[1], self.eps, self.wd)

    def state_dict(self) -> dict:
        return {"master": self.master, "m": self.m, "v": self.v, "step": self.step_count}
