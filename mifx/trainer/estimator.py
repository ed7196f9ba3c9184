"""Estimator-style training API used by Trainer user modules (`trainer_fn(hparams, schema)`).

Reference: `airflow-dags/taxi_utils.py:285-356` — `RunConfig(save_checkpoints_steps=999,
keep_checkpoint_max=1).replace(model_dir=serving_model_dir)`, `TrainSpec(input_fn, max_steps)`,
`EvalSpec(input_fn, steps, exporters=[FinalExporter('chicago-taxi', serving_receiver_fn)])`,
`DNNLinearCombinedClassifier(... warm_start_from=...)` and `train_and_evaluate`. Our estimator
trains on the fused gfx950 step when a GPU is visible (PyTorch reference path otherwise),
checkpoints to `model_dir` (safetensors, keep_checkpoint_max), and exports the
SavedModel-equivalent directories consumed by Evaluator / Pusher / serving.
"""
from __future__ import annotations

import dataclasses
import glob
import os
import time
from dataclasses import dataclass, field
from typing import Any, Callable

import numpy as np
import torch
from safetensors.torch import load_file, save_file

from ..models import wide_deep as wdm


@dataclass
class RunConfig:
    model_dir: str | None = None
    save_checkpoints_steps: int | None = 999
    keep_checkpoint_max: int = 1
    tf_random_seed: int = 0
    device: str | None = None

    def replace(self, **kw) -> "RunConfig":
        return dataclasses.replace(self, **kw)


@dataclass
class TrainSpec:
    input_fn: Callable
    max_steps: int


@dataclass
class EvalSpec:
    input_fn: Callable
    steps: int | None = None
    exporters: list = field(default_factory=list)
    name: str | None = None


@dataclass
class FinalExporter:
    name: str
    serving_input_receiver_fn: Callable

    def export(self, estimator, export_path: str) -> str:
        return estimator.export_saved_model(export_path, self.serving_input_receiver_fn)


class HParams:
    def __init__(self, **kw):
        self.__dict__.update(kw)

    def values(self) -> dict:
        return dict(self.__dict__)


def _dist_info() -> tuple[object, int, int]:
    """(process group, rank, world) when this process is one rank of a data-parallel Trainer
    (mifx.trainer.distributed), else (None, 0, 1)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.group.WORLD, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def _default_device(cfg: RunConfig) -> torch.device:
    dev = torch.device(cfg.device) if cfg.device else \
        (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    if dev.type == "cuda" and dev.index is None:  # one process per GPU: this rank's device
        shared = os.environ.get("MIFX_SHARED_GPU") == "1"  # multi-rank rehearsal on one GPU
        dev = torch.device("cuda", 0 if shared else int(os.environ.get("LOCAL_RANK", 0)))
    return dev


def shard_records(records: torch.Tensor, rank: int, world: int, batch: int) -> torch.Tensor:
    """Rank `rank`'s shard for data parallelism with per-replica batch `batch`: the records are cut into global
    batches of world * batch (remainder dropped) and rank r takes slice r of every global batch, so step i of
    the DP job trains on exactly the examples of step i of one process at batch world * batch."""
    g = world * batch
    n = records.shape[0] // g * g
    if n == 0:
        raise ValueError(f"{records.shape[0]} records < one global batch ({world} x {batch})")
    return records[:n].reshape(n // g, world, batch, *records.shape[1:])[:, rank].reshape(-1, *records.shape[1:]) \
        .contiguous()


def _auc(labels: np.ndarray, scores: np.ndarray) -> float:
    pos = labels > 0.5
    npos, nneg = int(pos.sum()), int((~pos).sum())
    if npos == 0 or nneg == 0:
        return float("nan")
    order = np.argsort(scores, kind="mergesort")
    ranks = np.empty(len(scores))
    ranks[order] = np.arange(1, len(scores) + 1)
    # average ranks for ties
    s = scores[order]
    i = 0
    while i < len(s):
        j = i
        while j + 1 < len(s) and s[j + 1] == s[i]:
            j += 1
        if j > i:
            ranks[order[i:j + 1]] = (i + j + 2) / 2.0
        i = j + 1
    return float((ranks[pos].sum() - npos * (npos + 1) / 2) / (npos * nneg))


class WideDeepEstimator:
    """DNNLinearCombinedClassifier equivalent for the taxi feature set."""

    def __init__(self, config: RunConfig, hidden_units: list[int] | None = None, warm_start_from: str | None = None,
                 batch_size: int = 40, loss_reduction: str = "sum", dnn_optimizer=None, linear_optimizer=None,
                 steps_per_graph: int = 100, shuffle: bool = True, eval_batch_size: int | None = None):
        """batch_size is per replica: a data-parallel Trainer with N ranks trains on N x batch_size examples per
        step (TF distributed Estimator semantics). steps_per_graph: training steps per hipGraph replay on the
        GPU (checkpoint boundaries and max_steps are honoured exactly; remainders replay a one-step graph).
        shuffle: a new pseudo-random order of the training records every epoch, seeded by
        config.tf_random_seed (`read_batch_features(randomize_input=True)`, `taxi_utils.py:275-276`); the same
        order on the CPU and GPU paths and for any number of data-parallel ranks (mifx.data.shuffle).
        eval_batch_size: the evaluation input's batch (default batch_size): evaluate(steps) reads steps x
        eval_batch_size examples, whatever the number of training ranks (`taxi_utils.py:304-305`: 40 / 40)."""
        self.config = config
        self.pg, self.rank, self.world = _dist_info()
        self.steps_per_graph = int(steps_per_graph)
        self.cfg = wdm.WideDeepConfig(hidden_units=list(hidden_units or wdm.dnn_hidden_units()))
        self.device = _default_device(config)
        self.batch_size = batch_size
        self.eval_batch_size = int(eval_batch_size or batch_size)
        self.loss_reduction = loss_reduction
        self.shuffle = bool(shuffle)
        self.dnn_optimizer, self.linear_optimizer = dnn_optimizer, linear_optimizer
        self.model = wdm.WideDeepModel(self.cfg, seed=config.tf_random_seed)
        self.global_step = 0
        if warm_start_from:
            self._load_weights(warm_start_from)
        elif config.model_dir and self.latest_checkpoint():
            self._restore(self.latest_checkpoint())
        self._trainer = None

    # ------------------------------------------------------------------ checkpoints
    def latest_checkpoint(self) -> str | None:
        if not self.config.model_dir:
            return None
        c = sorted(glob.glob(os.path.join(self.config.model_dir, "ckpt-*.safetensors")),
                   key=lambda p: int(p.rsplit("-", 1)[1].split(".")[0]))
        return c[-1] if c else None

    def _restore(self, path: str) -> None:
        """Model weights, the optimizer slots (canonical s0 / s1, either trainer's) and the global step."""
        sd = load_file(path)
        self.global_step = int(sd.pop("global_step").item()) if "global_step" in sd else 0
        self.model.load_state_dict({k: v for k, v in sd.items() if not k.startswith("opt.")}, strict=False)
        self._opt_state = {k[4:]: v for k, v in sd.items() if k.startswith("opt.")}

    def _load_weights(self, path: str) -> None:
        if os.path.isdir(path):
            cand = glob.glob(os.path.join(path, "**", "variables.safetensors"), recursive=True) or \
                glob.glob(os.path.join(path, "ckpt-*.safetensors"))
            path = sorted(cand)[-1]
        sd = load_file(path)
        self.model.load_state_dict({k: v for k, v in sd.items() if k in self.model.state_dict()}, strict=False)

    def _save_checkpoint(self) -> None:
        """Rank 0 writes ckpt-<step>.safetensors (weights, canonical optimizer slots, global step); every rank of
        a data-parallel job meets at a host barrier afterwards, so no replica waits on the device meanwhile."""
        d = self.config.model_dir
        tr = self._trainer
        if d and self.rank == 0:
            os.makedirs(d, exist_ok=True)
            sd = {k: v.detach().cpu().contiguous() for k, v in self.model.state_dict().items()}
            sd["global_step"] = torch.tensor([self.global_step], dtype=torch.int64)
            if tr is not None:
                st = tr.state_dict()
                sd["opt.s0"], sd["opt.s1"] = st["s0"].cpu().contiguous(), st["s1"].cpu().contiguous()
            save_file(sd, os.path.join(d, f"ckpt-{self.global_step}.safetensors"))
            self._prune_checkpoints(d)
        self._barrier()

    def _barrier(self) -> None:
        if self.pg is not None:
            torch.distributed.barrier(group=self.pg)

    def _prune_checkpoints(self, d: str) -> None:
        ck = sorted(glob.glob(os.path.join(d, "ckpt-*.safetensors")),
                    key=lambda p: int(p.rsplit("-", 1)[1].split(".")[0]))
        for old in ck[:-max(1, self.config.keep_checkpoint_max)]:
            os.remove(old)

    # ------------------------------------------------------------------ train / eval
    def _make_trainer(self, records: torch.Tensor):
        from .fused_wide_deep import FusedWideDeepTrainer, default_dnn_opt, default_wide_opt
        from .torch_wide_deep import TorchWideDeepTrainer

        dopt = self.dnn_optimizer or default_dnn_opt()
        wopt = self.linear_optimizer or default_wide_opt(len(self.cfg.wide))
        # every rank holds all records and reads its slice of one global stream (stride world x batch, offset
        # rank x batch): step i of a data-parallel job trains on exactly the examples of step i of one process at
        # batch world x batch, shuffled or not, and the ranks' rows are disjoint
        n = records.shape[0]
        bs = min(self.batch_size, n // self.world)
        if bs < 1:
            raise ValueError(f"{n} records < one global batch ({self.world} x {self.batch_size})")
        feed = dict(shuffle_seed=self.shuffle_seed() if self.shuffle else 0, feed_stride=self.world * bs,
                    feed_offset=self.rank * bs)
        if self.device.type == "cuda":
            tr = FusedWideDeepTrainer(self.model, batch=bs, device=self.device, dnn_opt=dopt, wide_opt=wopt,
                                      loss_reduction=self.loss_reduction, process_group=self.pg, **feed)
        else:
            tr = TorchWideDeepTrainer(self.model, batch=bs, device=self.device, dnn_opt=dopt, wide_opt=wopt,
                                      loss_reduction=self.loss_reduction, process_group=self.pg, **feed)
        st = getattr(self, "_opt_state", None) or {}
        tr.load_state_dict({"param": None, "s0": st.get("s0"), "s1": st.get("s1"),
                            "step": torch.tensor([self.global_step])})
        tr.set_data(records)
        return tr

    def shuffle_seed(self) -> int:
        """The (non-zero) shuffle key derived from config.tf_random_seed."""
        return ((int(self.config.tf_random_seed or 0) * 0x9E3779B97F4A7C15) ^ 0x5EEDF00D) % (2**64 - 1) + 1

    def _graph_setup(self, tr) -> None:
        """GPU: capture S-step hipGraphs (data-parallel: the xGMI exchange inside the graph, the direct RCCL
        path if its validation fails on any rank). The first steps already ran eagerly (lazy kernel / module
        initialisation), so capture runs no warmup steps of its own."""
        if self.pg is None:
            tr.capture(warmup=0, steps_per_graph=self.steps_per_graph)
            return
        ok = True
        try:
            tr.capture(warmup=0, steps_per_graph=self.steps_per_graph, dp_mode="xgmi")
        except Exception as e:  # noqa: BLE001 -- agreed on below
            import sys

            print(f"[estimator] xGMI exchange unavailable ({e}); using the RCCL path", file=sys.stderr)
            ok = False
        fdev = self.device if torch.distributed.get_backend(self.pg) == "nccl" else torch.device("cpu")
        flag = torch.tensor([0.0 if ok else 1.0], device=fdev)
        torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX, group=self.pg)
        if flag.item() != 0.0:
            tr.disable_xgmi()
            tr.capture(warmup=0, steps_per_graph=self.steps_per_graph, dp_mode="direct")

    def train(self, input_fn: Callable, max_steps: int, hooks: list | None = None) -> "WideDeepEstimator":
        """Train to global step `max_steps` (resuming from the latest checkpoint in model_dir), checkpointing
        every save_checkpoints_steps. On the GPU the steps between checkpoints run as multi-step hipGraph
        replays (per-step `hooks` force one host step at a time)."""
        records = input_fn()
        self._trainer = tr = self._make_trainer(records)
        every = self.config.save_checkpoints_steps or 0
        cuda = self.device.type == "cuda"
        t0, n0 = time.time(), self.global_step
        eager_first = 2  # lazy initialisation before any capture
        graphs = cuda and not hooks
        while self.global_step < max_steps:
            nxt = max_steps
            if every:
                nxt = min(nxt, (self.global_step // every + 1) * every)
            if hooks or (graphs and eager_first > 0):
                tr.step()
                self.global_step += 1
                eager_first -= 1
                for h in hooks or []:
                    h(self.global_step, tr)
                if graphs and eager_first == 0 and getattr(tr, "graph", None) is None:
                    self._graph_setup(tr)
            else:
                tr.run(nxt - self.global_step)
                self.global_step = nxt
            if every and self.global_step % every == 0:
                tr.sync_to_model()
                self._save_checkpoint()
        if cuda:
            torch.cuda.synchronize(self.device)
        self.train_seconds = time.time() - t0
        # whole-job rate: every replica trains batch examples per step
        self.examples_per_sec = (self.global_step - n0) * tr.batch * self.world / max(self.train_seconds, 1e-9)
        tr.sync_to_model()
        if not (every and self.global_step % every == 0):
            self._save_checkpoint()
        if hasattr(tr, "steps_done"):
            assert tr.steps_done == self.global_step, (tr.steps_done, self.global_step)
        return self

    def close(self) -> None:
        """Release the data-parallel exchange (collective: every rank calls it after train_and_evaluate)."""
        tr = self._trainer
        if tr is not None and getattr(tr, "_xg", None) is not None:
            tr.disable_xgmi()

    def predict_logits(self, records: torch.Tensor) -> np.ndarray:
        if self.device.type == "cuda":
            if self._trainer is None:
                self._trainer = self._make_trainer(records)
            return self._trainer.predict_logits(records).cpu().numpy()
        dense, ids, _ = wdm.records_to_tensors(records)
        with torch.no_grad():
            return self.model(dense, ids).numpy()

    def evaluate(self, input_fn: Callable, steps: int | None = None, name: str | None = None) -> dict:
        records = input_fn()
        # `steps` batches of the input batch size, whatever the number of training ranks (TF Estimator evaluate:
        # the evaluator runs eval_spec.steps batches of its input_fn's batch size)
        n = records.shape[0] if not steps else min(records.shape[0], steps * self.eval_batch_size)
        records = records[:n]
        logits = self.predict_logits(records)
        _, _, label = wdm.records_to_tensors(records.cpu())
        y = label.numpy()
        p = 1.0 / (1.0 + np.exp(-logits))
        loss = np.maximum(logits, 0) - logits * y + np.log1p(np.exp(-np.abs(logits)))
        m = {"loss": float(loss.mean() * self.eval_batch_size), "average_loss": float(loss.mean()),
             "accuracy": float(((p > 0.5) == (y > 0.5)).mean()), "auc": _auc(y, p),
             "prediction/mean": float(p.mean()), "label/mean": float(y.mean()), "global_step": self.global_step}
        self.last_eval = m
        if self.config.model_dir:
            import json

            d = os.path.join(self.config.model_dir, f"eval_{name or 'default'}")
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, "metrics.json"), "w") as f:
                json.dump(m, f)
        return m

    # ------------------------------------------------------------------ export
    def export_saved_model(self, export_dir_base: str, serving_input_receiver_fn: Callable | None = None) -> str:
        from ..serving import saved_model

        receiver = serving_input_receiver_fn() if serving_input_receiver_fn else {}
        path = os.path.join(export_dir_base, str(int(time.time() * 1000)))
        saved_model.save_wide_deep(path, self.model, receiver, global_step=self.global_step)
        return path

    export_savedmodel = export_saved_model


def train_and_evaluate(estimator, train_spec: TrainSpec, eval_spec: EvalSpec) -> tuple[dict, list[str]]:
    """Data-parallel ranks all train; rank 0 alone evaluates and exports (the others return ({}, []))."""
    estimator.train(train_spec.input_fn, max_steps=train_spec.max_steps)
    if getattr(estimator, "rank", 0) != 0:
        return {}, []
    metrics = estimator.evaluate(eval_spec.input_fn, steps=eval_spec.steps, name=eval_spec.name)
    exports = []
    for ex in eval_spec.exporters:
        base = os.path.join(estimator.config.model_dir or ".", "export", ex.name)
        exports.append(ex.export(estimator, base))
    return metrics, exports


__all__ = ["RunConfig", "TrainSpec", "EvalSpec", "FinalExporter", "HParams", "WideDeepEstimator",
           "train_and_evaluate", "shard_records", "Any"]
