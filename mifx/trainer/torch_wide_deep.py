"""Portable PyTorch Wide&Deep trainer (CPU reference path; same optimizers/semantics as the
fused HIP trainer). Used by the Trainer component on CPU-only hosts and as the numerics oracle
in tests.

Checkpoint state uses the fused trainer's canonical layout (`state_dict()`: param / s0 / s1 vectors
[WTOT + NWIDE] + step), so a checkpoint written on one path resumes on the other: s0 / s1 are the
Adagrad accumulator, FTRL (accumulator, linear) and Adam (m, v) slots of csrc/wide_deep.hip
opt_update."""
from __future__ import annotations

import copy

import numpy as np
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
                 process_group=None, shuffle_seed: int = 0, feed_stride: int | None = None, feed_offset: int = 0):
        """shuffle_seed / feed_stride / feed_offset: the record stream of the fused GPU trainer (csrc/feed.h,
        mifx.data.shuffle): the same records per step, so both paths train on identical batches."""
        self.device = torch.device(device)
        self.model = (model or wdm.WideDeepModel()).to(self.device)
        # DP: "sum" losses are summed across ranks (global-batch sum, like the fused trainer); "mean"
        # losses are averaged, i.e. the mean over the global batch
        self.dp = DataParallel(self.model, process_group, average=(loss_reduction == "mean")) \
            if process_group is not None else None
        self.batch = batch
        self.shuffle_seed = int(shuffle_seed)
        self.feed_stride = int(feed_stride) if feed_stride is not None else int(batch)
        self.feed_offset = int(feed_offset)
        self.loss_reduction = loss_reduction
        dnn_params = [p for n, p in self.model.named_parameters() if not n.startswith("wide")]
        wide_params = [self.model.wide, self.model.wide_bias]
        dspec, wspec = dnn_opt or default_dnn_opt(), wide_opt or default_wide_opt(len(self.model.cfg.wide))
        self.opt_dnn = _mk(dspec, dnn_params)
        self.opt_wide = _mk(wspec, wide_params)
        self.dnn_kind, self.wide_kind = dspec.kind, wspec.kind
        # initial slot values (what the fused trainer starts s0 / s1 at)
        self._init = [(spec.initial_accumulator_value if spec.kind in ("adagrad", "ftrl") else 0.0, 0.0)
                      for spec in (dspec, wspec)]
        self.records = None
        self.step_idx = 0
        self._last_loss = float("nan")

    def set_data(self, records: torch.Tensor) -> None:
        dense, ids, label = wdm.records_to_tensors(records.cpu())
        self.dense, self.ids, self.label = dense.to(self.device), ids.to(self.device), label.to(self.device)
        self.n_data = len(label)
        self.records = records

    def _batch_idx(self) -> torch.Tensor:
        from ..data.shuffle import record_indices

        idx = record_indices(self.step_idx, self.batch, self.n_data, self.feed_stride, self.feed_offset,
                             self.shuffle_seed)
        return torch.from_numpy(idx).to(self.device)

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

    def run(self, n: int) -> None:
        for _ in range(n):
            self.step()

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

    # ---------------------------------------------------------------- checkpoint state (canonical layout)
    _SLOTS = {"adagrad": ("acc", None), "ftrl": ("acc", "lin"), "adam": ("exp_avg", "exp_avg_sq"), "sgd": (None, None)}

    def _opts(self):
        return ((self.opt_dnn, self.dnn_kind, lambda n: not n.startswith("wide"), self._init[0]),
                (self.opt_wide, self.wide_kind, lambda n: n.startswith("wide"), self._init[1]))

    def _slot_vectors(self) -> tuple[np.ndarray, np.ndarray]:
        """Optimizer slots as canonical vectors (parameters without state yet hold the slot's initial value)."""
        out = []
        for slot in (0, 1):
            m = copy.deepcopy(self.model).cpu()
            with torch.no_grad():
                for (opt, kind, sel, inits) in self._opts():
                    key = self._SLOTS[kind][slot]
                    init = inits[slot]
                    for (n, p), (_, q) in zip(self.model.named_parameters(), m.named_parameters()):
                        if not sel(n):
                            continue
                        st = opt.state.get(p, {})
                        q.copy_(st[key].cpu() if key in st else torch.full_like(q, init))
            out.append(wdm.pack_canonical(m))
        return out[0], out[1]

    def state_dict(self) -> dict:
        s0, s1 = self._slot_vectors()
        return {"param": torch.from_numpy(wdm.pack_canonical(self.model)), "s0": torch.from_numpy(s0),
                "s1": torch.from_numpy(s1), "step": torch.tensor([self.step_idx], dtype=torch.int64)}

    def load_state_dict(self, sd: dict) -> None:
        if sd.get("param") is not None:
            wdm.unpack_canonical(sd["param"], self.model)
        if "step" in sd:
            self.step_idx = int(torch.as_tensor(sd["step"]).reshape(-1)[0])
        slots = [sd.get("s0"), sd.get("s1")]
        views = []
        for v in slots:
            if v is None:
                views.append(None)
                continue
            m = copy.deepcopy(self.model).cpu()
            wdm.unpack_canonical(v, m)
            views.append(dict(m.named_parameters()))
        for (opt, kind, sel, _) in self._opts():
            for n, p in self.model.named_parameters():
                if not sel(n):
                    continue
                st = opt.state[p]
                for slot in (0, 1):
                    key = self._SLOTS[kind][slot]
                    if key is None or views[slot] is None:
                        continue
                    st[key] = views[slot][n].detach().clone().to(p.device)
                if kind == "ftrl" and "lin" not in st:
                    st["lin"] = torch.zeros_like(p)
                if kind == "adam":
                    st.setdefault("exp_avg", torch.zeros_like(p))
                    st.setdefault("exp_avg_sq", torch.zeros_like(p))
                    st["step"] = torch.tensor(float(self.step_idx))
