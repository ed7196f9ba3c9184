"""Trainer for the KFP taxi DNN (`mifx.models.taxi_dnn`): HIP gather/scatter kernels on GPU,
PyTorch autograd + TF-semantics Adagrad on CPU (the numerics oracle).

Reference: dnntrainer component (`taxi-cab-classification-pipeline.py:117-126`): Adagrad lr 0.1,
hidden 1500, 3,000 steps, binary head; TF's Adagrad starts accumulators at 0.1."""
from __future__ import annotations

import numpy as np
import torch

from ..models.taxi_dnn import TaxiDNN
from .optim import TFAdagrad


class TaxiDNNTrainer:
    def __init__(self, model: TaxiDNN | None = None, batch: int = 32, lr: float = 0.1, device="cpu",
                 initial_accumulator_value: float = 0.1, loss_reduction: str = "sum", native: bool | None = None):
        self.device = torch.device(device)
        self.model = (model or TaxiDNN()).to(self.device)
        self.batch, self.lr, self.loss_reduction = batch, lr, loss_reduction
        self.native = (self.device.type == "cuda") if native is None else native
        self.dense_row0 = self.model.cfg.sparse_rows
        if self.native:
            from ..ops import embag_mlp

            self._k = embag_mlp
            p = {n: getattr(self.model, n) for n in ("W1", "b1", "w2", "b2")}
            self.params = {n: t.data for n, t in p.items()}
            self.accs = {n: torch.full_like(t, initial_accumulator_value) for n, t in self.params.items()}
            self.bufs = embag_mlp.make_buffers(batch, self.model.cfg.hidden, len(self.model.cfg.dense), self.device)
        else:
            self.opt = TFAdagrad(self.model.parameters(), lr=lr, initial_accumulator_value=initial_accumulator_value)
        self.step_idx = 0
        self._last = float("nan")

    def set_data(self, ids: torch.Tensor, dense: torch.Tensor, label: torch.Tensor) -> None:
        self.rows = self.model.rows(ids.to(self.device)).to(torch.int32).contiguous()
        self.dense = dense.to(self.device).float().contiguous()
        self.label = label.to(self.device).float().contiguous()
        self.n = len(self.label)

    def _idx(self):
        s = (self.step_idx * self.batch) % self.n
        return (torch.arange(self.batch, device=self.device) + s) % self.n

    def step(self) -> None:
        idx = self._idx()
        rows, xd, y = self.rows[idx].contiguous(), self.dense[idx].contiguous(), self.label[idx].contiguous()
        if self.native:
            scale = 1.0 if self.loss_reduction == "sum" else 1.0 / self.batch
            self._k.fwd_bwd(self.params["W1"], self.params["b1"], self.params["w2"], self.params["b2"], rows, xd, y,
                            self.dense_row0, scale, True, self.bufs)
            self._k.adagrad(self.params, self.accs, rows, xd, self.dense_row0, self.bufs, self.lr)
            self._last_t = self.bufs["loss"]
        else:
            logit = self._forward_rows(rows, xd)
            loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, y, reduction=self.loss_reduction)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            self.opt.step()
            self._last = float(loss.detach()) * (self.batch if self.loss_reduction == "mean" else 1.0)
        self.step_idx += 1

    def last_loss(self) -> float:
        if self.native:
            return float(self._last_t.sum())
        return self._last

    @torch.no_grad()
    def predict_logits(self, ids: torch.Tensor, dense: torch.Tensor, batch: int = 4096) -> np.ndarray:
        out = []
        for s in range(0, len(ids), batch):
            r = self.model.rows(ids[s:s + batch].to(self.device)).to(torch.int32).contiguous()
            xd = dense[s:s + batch].to(self.device).float().contiguous()
            if self.native:
                bufs = self._k.make_buffers(len(r), self.model.cfg.hidden, xd.shape[1], self.device)
                self._k.fwd_bwd(self.params["W1"], self.params["b1"], self.params["w2"], self.params["b2"], r, xd,
                                bufs["logit"], self.dense_row0, 1.0, False, bufs)
                out.append(bufs["logit"].cpu())
            else:
                out.append(self._forward_rows(r, xd).cpu())
        return torch.cat(out).numpy()

    def _forward_rows(self, rows: torch.Tensor, xd: torch.Tensor) -> torch.Tensor:
        """Reference forward on global W1 rows (what the HIP kernel computes)."""
        m = self.model
        z = m.b1 + m.W1[rows.long()].sum(1) + xd @ m.W1[self.dense_row0:]
        return torch.relu(z) @ m.w2 + m.b2
