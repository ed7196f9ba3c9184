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
    """On the GPU a step is 5 HIP launches with no host work: the batch is selected on the device from the
    HBM-resident records through a device step counter (advanced by the optimizer kernel), and the sparse Adagrad
    deduplicates rows in-kernel (no sort/unique, whose dynamic output size synchronised the host every step). So
    the step is captured once into hipGraphs -- one step and `steps_per_graph` consecutive steps -- and replayed
    (`graph=False`: eager launches of the same kernels)."""

    def __init__(self, model: TaxiDNN | None = None, batch: int = 32, lr: float = 0.1, device="cpu",
                 initial_accumulator_value: float = 0.1, loss_reduction: str = "sum", native: bool | None = None,
                 graph: bool = True, steps_per_graph: int = 50):
        self.device = torch.device(device)
        self.model = (model or TaxiDNN()).to(self.device)
        self.batch, self.lr, self.loss_reduction = batch, lr, loss_reduction
        self.native = (self.device.type == "cuda") if native is None else native
        self.dense_row0 = self.model.cfg.sparse_rows
        self.use_graph = bool(graph and self.native)
        self.steps_per_graph = max(1, int(steps_per_graph))
        self.graph, self.graph_multi = None, None
        if self.native:
            from ..ops import embag_mlp

            self._k = embag_mlp
            if batch > embag_mlp.limits()["max_batch"]:
                raise ValueError(f"batch {batch} > {embag_mlp.limits()['max_batch']} (csrc/embag_mlp.hip kMaxList)")
            self.step_ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
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
        if self.n < self.batch:
            raise ValueError(f"{self.n} records < batch {self.batch}")
        if self.native:  # the device counter continues from the host's step count
            self.step_ctr.fill_(self.step_idx)
        # captured graphs hold the previous tensors' addresses and record count: recapture on the next step
        self.graph, self.graph_multi = None, None

    def _idx(self):
        s = (self.step_idx * self.batch) % self.n
        return (torch.arange(self.batch, device=self.device) + s) % self.n

    def _native_step(self) -> None:
        scale = 1.0 if self.loss_reduction == "sum" else 1.0 / self.batch
        p = self.params
        self._k.fwd_bwd(p["W1"], p["b1"], p["w2"], p["b2"], self.rows, self.dense, self.label, self.dense_row0, scale,
                        True, self.bufs, batch=self.batch, step_ctr=self.step_ctr)
        self._k.adagrad(p, self.accs, self.rows, self.dense, self.dense_row0, self.bufs, self.lr, batch=self.batch,
                        step_ctr=self.step_ctr)

    def capture(self) -> None:
        """Capture one step and `steps_per_graph` consecutive steps as hipGraphs (every captured step reads the
        device counter, so replays walk through the data and the optimizer state like eager steps)."""
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._native_step()
        gm = None
        if self.steps_per_graph > 1:
            gm = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm):
                for _ in range(self.steps_per_graph):
                    self._native_step()
        self.graph, self.graph_multi = g, gm

    def run(self, n: int) -> None:
        """n training steps: the first eagerly (lazy library/kernel initialisation), then multi-step graph replays
        and single-step replays for the remainder."""
        while n > 0 and self.use_graph and self.graph is None:
            self.step()  # step() captures once a first eager step has run
            n -= 1
        if self.graph_multi is not None:
            reps, n = divmod(n, self.steps_per_graph)
            for _ in range(reps):
                self.graph_multi.replay()
                self.step_idx += self.steps_per_graph
        for _ in range(n):
            self.step()

    def step(self) -> None:
        if self.native:
            if self.use_graph and self.graph is None and self.step_idx >= 1:  # first step eager (lazy init), then
                self.capture()
            if self.graph is not None:
                self.graph.replay()
            else:
                self._native_step()
            self._last_t = self.bufs["loss"]
        else:
            idx = self._idx()
            rows, xd, y = self.rows[idx].contiguous(), self.dense[idx].contiguous(), self.label[idx].contiguous()
            logit = self._forward_rows(rows, xd)
            loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, y, reduction=self.loss_reduction)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            self.opt.step()
            self._last = float(loss.detach()) * (self.batch if self.loss_reduction == "mean" else 1.0)
        self.step_idx += 1

    def last_loss(self) -> float:
        if self.native:
            return float(self.bufs["loss"].sum())
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
