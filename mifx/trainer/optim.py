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
