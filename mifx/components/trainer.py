"""Trainer, Evaluator, ModelValidator and Pusher components.

Reference (`airflow-dags/taxi_pipeline.py:92-120`):
* `Trainer(module_file, transformed_examples, schema, transform_output, train_args=TrainArgs(num_steps=10000),
  eval_args=EvalArgs(num_steps=5000))` calls `trainer_fn(hparams, schema)` (`taxi_utils.py:285-356`) with
  hparams.{train_files, eval_files, transform_output, train_steps, eval_steps, serving_model_dir,
  warm_start_from}; outputs `serving_model_dir/export/<exporter>/<ts>` and `eval_model_dir/<ts>`.
* `Evaluator(examples, model_exports, feature_slicing_spec)` -> sliced metrics (ModelEvalPath).
* `ModelValidator(examples, model)` -> blessing vs the last blessed model (ModelBlessingPath).
* `Pusher(model_export, model_blessing, push_destination=Filesystem(base_directory))` -> versioned copy.
"""
from __future__ import annotations

import json
import os
import shutil
import time

import numpy as np

from ..evaluator import metrics as em
from ..io import dataset
from ..orchestration import artifact as A
from ..orchestration.component import BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec, ExecutionParameter
from ..serving import saved_model
from . import proto
from .statistics import load_schema_from_artifact
from .transform import table_to_inputs

SERVING_DIR = "serving_model_dir"
EVAL_DIR = "eval_model_dir"


# -------------------------------------------------------------------------------- Trainer
class TrainerSpec(ComponentSpec):
    PARAMETERS = {"module_file": ExecutionParameter(), "train_args": ExecutionParameter(),
                  "eval_args": ExecutionParameter(), "custom_config": ExecutionParameter(optional=True),
                  "warm_start": ExecutionParameter(optional=True, default=False)}
    INPUTS = {"transformed_examples": ChannelParameter(A.EXAMPLES), "schema": ChannelParameter(A.SCHEMA),
              "transform_output": ChannelParameter(A.TRANSFORM, optional=True)}
    OUTPUTS = {"output": ChannelParameter(A.MODEL)}


class TrainerExecutor(BaseExecutor):
    """custom_config["num_gpus"] = N > 1 trains data-parallel: N ranks (one per GPU; gloo processes on a CPU
    host) launched by mifx.trainer.distributed, each running the same trainer_fn on its shard of every global
    batch; rank 0 evaluates and exports. Otherwise trainer_fn runs in this process."""

    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        ex = {a.split: a.uri for a in input_dict["transformed_examples"]}
        out = output_dict["output"][0]
        targs = proto.from_dict(proto.TrainArgs, exec_properties["train_args"])
        eargs = proto.from_dict(proto.EvalArgs, exec_properties["eval_args"])
        custom = dict(exec_properties.get("custom_config") or {})
        hp = dict(train_files=[ex.get("train", next(iter(ex.values())))], eval_files=[ex.get("eval", "")],
                  transform_output=input_dict["transform_output"][0].uri if input_dict.get("transform_output")
                  else None, train_steps=targs.num_steps, eval_steps=eargs.num_steps,
                  serving_model_dir=os.path.join(out.uri, SERVING_DIR),
                  eval_model_dir=os.path.join(out.uri, EVAL_DIR), warm_start_from=custom.get("warm_start_from"),
                  device=self.context.device, custom_config=custom)
        module_file, schema_uri = exec_properties["module_file"], input_dict["schema"][0].uri
        n = int(custom.get("num_gpus", 1) or 1)
        if n > 1:
            from ..trainer import distributed

            res = distributed.launch({"module_file": module_file, "hparams": hp, "schema_uri": schema_uri,
                                      "out_dir": out.uri, "work_dir": os.path.join(out.uri, "dp_run")},
                                     n, os.path.join(out.uri, "dp_run"), timeout=custom.get("timeout_s"))
        else:
            from ..trainer.distributed import run_trainer_fn

            res = run_trainer_fn(module_file, hp, schema_uri, out.uri)
        metrics = res["eval"]
        with open(os.path.join(out.uri, "metrics.json"), "w") as f:
            json.dump(res, f, default=float)
        out.custom_properties["train_steps"] = int(targs.num_steps)
        out.custom_properties["num_replicas"] = int(res.get("world_size") or 1)
        if res.get("train_examples_per_sec"):
            out.custom_properties["train_examples_per_sec"] = float(res["train_examples_per_sec"])
        for k in ("accuracy", "auc", "average_loss"):
            if k in metrics and metrics[k] == metrics[k]:
                out.custom_properties[f"eval_{k}"] = float(metrics[k])


class Trainer(BaseComponent):
    SPEC_CLASS = TrainerSpec
    EXECUTOR_CLASS = TrainerExecutor
    EXECUTION_TYPE = "trainer"

    def __init__(self, module_file: str, transformed_examples, schema, train_args, eval_args,
                 transform_output=None, custom_config: dict | None = None, name: str | None = None, output=None):
        super().__init__(TrainerSpec(module_file=os.path.abspath(module_file), transformed_examples=transformed_examples,
                                     schema=schema, transform_output=transform_output,
                                     train_args=train_args.to_dict() if hasattr(train_args, "to_dict") else train_args,
                                     eval_args=eval_args.to_dict() if hasattr(eval_args, "to_dict") else eval_args,
                                     custom_config=custom_config, output=output), name=name)


def latest_model_dir(model_uri: str, kind: str = EVAL_DIR) -> str:
    base = os.path.join(model_uri, kind)
    if kind == SERVING_DIR:
        exp = os.path.join(base, "export")
        names = sorted(os.listdir(exp))
        return saved_model.latest_export(os.path.join(exp, names[-1]))
    return saved_model.latest_export(base)


def _eval_predictions(model_uri: str, examples_uri: str):
    """Run the eval model over raw examples: returns (labels, probabilities, raw feature columns)."""
    loaded = saved_model.load(latest_model_dir(model_uri, EVAL_DIR))
    raw = table_to_inputs(dataset.read_split(examples_uri))
    label_key = loaded.meta["receiver"]["label_key"]
    tcols = loaded.transform.transform_raw_features(raw) if loaded.transform else raw
    labels = np.asarray(tcols[label_key], np.float64)
    logits = loaded.wd_logits(raw)
    return labels, 1.0 / (1.0 + np.exp(-logits)), raw


# ------------------------------------------------------------------------------ Evaluator
class EvaluatorSpec(ComponentSpec):
    PARAMETERS = {"feature_slicing_spec": ExecutionParameter(optional=True)}
    INPUTS = {"examples": ChannelParameter(A.EXAMPLES), "model_exports": ChannelParameter(A.MODEL)}
    OUTPUTS = {"output": ChannelParameter(A.MODEL_EVAL)}


class EvaluatorExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        ex = {a.split: a.uri for a in input_dict["examples"]}
        model_uri = input_dict["model_exports"][0].uri
        y, p, raw = _eval_predictions(model_uri, ex.get("eval", next(iter(ex.values()))))
        fss = proto.from_dict(proto.FeatureSlicingSpec, exec_properties.get("feature_slicing_spec")) or \
            proto.FeatureSlicingSpec()
        specs = [em.SliceSpec(columns=list(s.column_for_slicing)) for s in fss.specs]
        res = em.compute_sliced_metrics(y, p, raw, specs, device=self.context.device)
        res.model_location, res.data_location = model_uri, ex.get("eval", "")
        out = output_dict["output"][0]
        em.save_eval_result(res, out.uri)
        for k, v in res.overall().items():
            if isinstance(v, float) and v == v:
                out.custom_properties[k.replace("/", "_")] = v


class Evaluator(BaseComponent):
    SPEC_CLASS = EvaluatorSpec
    EXECUTOR_CLASS = EvaluatorExecutor
    EXECUTION_TYPE = "evaluator"

    def __init__(self, examples, model_exports, feature_slicing_spec=None, name: str | None = None, output=None):
        fss = feature_slicing_spec.to_dict() if hasattr(feature_slicing_spec, "to_dict") else feature_slicing_spec
        super().__init__(EvaluatorSpec(examples=examples, model_exports=model_exports, feature_slicing_spec=fss,
                                       output=output), name=name)


# ------------------------------------------------------------------------- ModelValidator
class ModelValidatorSpec(ComponentSpec):
    PARAMETERS = {"metric": ExecutionParameter(optional=True, default="auc"),
                  "tolerance": ExecutionParameter(optional=True, default=0.0)}
    INPUTS = {"examples": ChannelParameter(A.EXAMPLES), "model": ChannelParameter(A.MODEL)}
    OUTPUTS = {"blessing": ChannelParameter(A.MODEL_BLESSING)}


class ModelValidatorExecutor(BaseExecutor):
    def _last_blessed(self):
        store = self.context.extra.get("__metadata_store__")
        if store is None:
            return None
        for a in reversed(store.get_artifacts_by_type(A.MODEL_BLESSING)):
            if a.custom_properties["blessed"].int_value == 1:
                return a.custom_properties["current_model"].string_value, \
                    a.custom_properties["current_model_id"].int_value
        return None

    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        ex = {a.split: a.uri for a in input_dict["examples"]}
        eval_uri = ex.get("eval", next(iter(ex.values())))
        cand = input_dict["model"][0]
        metric = exec_properties.get("metric") or "auc"
        tol = float(exec_properties.get("tolerance") or 0.0)
        dev = self.context.device

        def score(y, p):  # overall metric: one GPU segmented reduction on a device, else the host pass
            return em.compute_sliced_metrics(y, p, {}, None, device=dev).overall()[metric]

        y, p, _ = _eval_predictions(cand.uri, eval_uri)
        cur = score(y, p)
        out = output_dict["blessing"][0]
        prev = self._last_blessed()
        blessed, base = True, None
        if prev is not None and os.path.exists(prev[0]):
            yb, pb, _ = _eval_predictions(prev[0], eval_uri)
            base = score(yb, pb)
            lower_is_better = metric in ("average_loss", "loss")
            blessed = cur <= base + tol if lower_is_better else cur >= base - tol
        with open(os.path.join(out.uri, "BLESSED" if blessed else "NOT_BLESSED"), "w") as f:
            json.dump({"metric": metric, "candidate": cur, "baseline": base}, f)
        out.custom_properties.update(blessed=int(blessed), current_model=cand.uri, current_model_id=int(cand.id or 0),
                                     candidate_metric=float(cur))
        if prev is not None:
            out.custom_properties.update(blessed_model=prev[0], blessed_model_id=int(prev[1]))


class ModelValidator(BaseComponent):
    SPEC_CLASS = ModelValidatorSpec
    EXECUTOR_CLASS = ModelValidatorExecutor
    EXECUTION_TYPE = "model_validator"

    def __init__(self, examples, model, metric: str = "auc", tolerance: float = 0.0, name: str | None = None,
                 blessing=None):
        super().__init__(ModelValidatorSpec(examples=examples, model=model, metric=metric, tolerance=tolerance,
                                            blessing=blessing), name=name)


# --------------------------------------------------------------------------------- Pusher
class PusherSpec(ComponentSpec):
    PARAMETERS = {"push_destination": ExecutionParameter()}
    INPUTS = {"model_export": ChannelParameter(A.MODEL), "model_blessing": ChannelParameter(A.MODEL_BLESSING)}
    OUTPUTS = {"model_push": ChannelParameter(A.PUSHED_MODEL)}


class PusherExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        out = output_dict["model_push"][0]
        bless = input_dict["model_blessing"][0]
        if not os.path.exists(os.path.join(bless.uri, "BLESSED")):
            out.custom_properties["pushed"] = 0
            return
        dest = proto.from_dict(proto.PushDestination, exec_properties["push_destination"])
        src = latest_model_dir(input_dict["model_export"][0].uri, SERVING_DIR)
        version = str(int(time.time()))
        target = os.path.join(dest.filesystem.base_directory, version)
        while os.path.exists(target):
            version = str(int(version) + 1)
            target = os.path.join(dest.filesystem.base_directory, version)
        shutil.copytree(src, target)
        shutil.copytree(src, out.uri, dirs_exist_ok=True)
        out.custom_properties.update(pushed=1, pushed_model=target, pushed_model_version=version)


class Pusher(BaseComponent):
    SPEC_CLASS = PusherSpec
    EXECUTOR_CLASS = PusherExecutor
    EXECUTION_TYPE = "pusher"

    def __init__(self, model_export, model_blessing, push_destination, name: str | None = None, model_push=None):
        pd_ = push_destination.to_dict() if hasattr(push_destination, "to_dict") else push_destination
        super().__init__(PusherSpec(model_export=model_export, model_blessing=model_blessing, push_destination=pd_,
                                    model_push=model_push), name=name)
