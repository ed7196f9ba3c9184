"""Portable PyTorch Wide&Deep trainer (CPU reference path; same optimizers/semantics as the
fused HIP trainer). Used by the Trainer component on CPU-only hosts and as the numerics oracle
in tests."""
from __future__ import annotations

import torch

from ..models import wide_deep as wdm
from ..parallel.ddp import DataParallel
from .fused_wide_deep import OptSpec, default_dnn_opt, default_wide_opt
from .optim import make_optimizer


def _mk(spec: OptSpec, params):
    kw = {}
    if spec.kind in ("adagrad", "ftrl"):
        kw["initial_accumulator_value"] = spec.initial_accumulator_value
    if spec.kind == "ftrl":
        kw.update(lr_power=spec.lr_power, l1=spec.l1, l2=spec.l2)
    if spec.kind == "adam":
        kw.update(betas=(spec.beta1, spec.beta2), eps=spec.eps)
    return make_optimizer(spec.kind, params, spec.lr, **kw)


class TorchWideDeepTrainer:
    def __init__(self, model: wdm.WideDeepModel | None = None, batch: int = 40, device="cpu",
                 dnn_opt: OptSpec | None = None, wide_opt: OptSpec | None = None, loss_reduction: str = "sum",
                 process_group=None):
        self.device = torch.device(device)
        self.model = (model or wdm.WideDeepModel()).to(self.device)
        # DP: "sum" losses are summed across ranks (global-batch sum, like the fused trainer); "mean"
        # losses are averaged, i.e. the mean over the global batch
        self.dp = DataParallel(self.model, process_group, average=(loss_reduction == "mean")) \
            if process_group is not None else None
        self.batch = batch
        self.loss_reduction = loss_reduction
        dnn_params = [p for n, p in self.model.named_parameters() if not n.startswith("wide")]
        wide_params = [self.model.wide, self.model.wide_bias]
        self.opt_dnn = _mk(dnn_opt or default_dnn_opt(), dnn_params)
        self.opt_wide = _mk(wide_opt or default_wide_opt(len(self.model.cfg.wide)), wide_params)
        self.records = None
        self.step_idx = 0
        self._last_loss = float("nan")

    def set_data(self, records: torch.Tensor) -> None:
        dense, ids, label = wdm.records_to_tensors(records.cpu())
        self.dense, self.ids, self.label = dense.to(self.device), ids.to(self.device), label.to(self.device)
        self.n_data = len(label)
        self.records = records

    def _batch_idx(self) -> torch.Tensor:
        start = (self.step_idx * self.batch) % self.n_data
        return (torch.arange(self.batch, device=self.device) + start) % self.n_data

    def step(self) -> None:
        idx = self._batch_idx()
        loss = self.model.loss(self.dense[idx], self.ids[idx], self.label[idx], reduction=self.loss_reduction)
        self.opt_dnn.zero_grad(set_to_none=True)
        self.opt_wide.zero_grad(set_to_none=True)
        loss.backward()
        if self.dp is not None:
            self.dp.finish()
        self.opt_dnn.step()
        self.opt_wide.step()
        self.step_idx += 1
        self._last_loss = float(loss.detach()) * (self.batch if self.loss_reduction == "mean" else 1.0)

    def last_loss(self) -> float:
        return self._last_loss

    @property
    def steps_done(self) -> int:
        return self.step_idx

    @torch.no_grad()
    def predict_logits(self, records: torch.Tensor) -> torch.Tensor:
        dense, ids, _ = wdm.records_to_tensors(records.cpu())
        return self.model(dense.to(self.device), ids.to(self.device))

    def sync_to_model(self) -> wdm.WideDeepModel:
        return self.model
