"""SavedModel-equivalent export format and loader.

Layout (mirrors TF's `<export_dir_base>/<timestamp>/` versioned exports consumed by TF Serving,
`Predict_Fashion_MNIST.ipynb:L189` and `taxi_utils.py:326,348-356`)::

    <dir>/saved_model.json            format, model family/class/config, signatures, receiver
    <dir>/variables/variables.safetensors
    <dir>/assets/transform/...        copy of the Transform graph (serving/eval receivers)

Families: ``wide_deep`` (taxi W&D; raw-example receiver through the Transform graph, classify
outputs) and ``module`` (any torch.nn.Module given by ``module_class`` + config, tensor inputs).
"""
from __future__ import annotations

import importlib
import json
import os
import shutil

import numpy as np
import torch
from safetensors.torch import load_file, save_file

FORMAT = "mifx.saved_model/v1"


def _write(path: str, meta: dict, state_dict: dict) -> None:
    os.makedirs(os.path.join(path, "variables"), exist_ok=True)
    save_file({k: v.detach().cpu().contiguous() for k, v in state_dict.items()},
              os.path.join(path, "variables", "variables.safetensors"))
    with open(os.path.join(path, "saved_model.json"), "w") as f:
        json.dump(meta, f, indent=1)


def save_wide_deep(path: str, model, receiver: dict | None = None, global_step: int = 0) -> str:
    receiver = dict(receiver or {})
    tdir = receiver.pop("transform_output", None)
    if tdir:
        dst = os.path.join(path, "assets", "transform")
        shutil.copytree(tdir, dst, dirs_exist_ok=True)
    meta = {"format": FORMAT, "family": "wide_deep", "global_step": global_step,
            "model_class": "mifx.models.wide_deep:WideDeepModel",
            "model_config": {"hidden_units": list(model.cfg.hidden_units), "wide": [list(x) for x in model.cfg.wide],
                             "dense_features": list(model.cfg.dense_features), "label": model.cfg.label},
            "receiver": {"kind": receiver.get("kind", "transformed"), "has_transform": bool(tdir),
                         "raw_label_key": receiver.get("raw_label_key"),
                         "label_key": receiver.get("label_key", model.cfg.label)},
            "signatures": {"serving_default": {"method": "classify", "inputs": receiver.get("raw_feature_spec", {}),
                                               "outputs": ["logits", "logistic", "probabilities", "class_ids",
                                                           "classes"]}}}
    _write(path, meta, model.state_dict())
    return path


def save_module(path: str, model: torch.nn.Module, module_class: str, config: dict | None = None,
                input_shape: list | None = None, class_names: list | None = None) -> str:
    meta = {"format": FORMAT, "family": "module", "model_class": module_class, "model_config": config or {},
            "signatures": {"serving_default": {"method": "predict", "inputs": {"input": input_shape},
                                               "outputs": ["scores"], "class_names": class_names}}}
    _write(path, meta, model.state_dict())
    return path


# Model classes a "module" export may name. An export is data (JSON + safetensors); the class it names is imported and
# called with the export's model_config as keyword arguments, so an open set of classes would let whoever writes an
# export (or uploads one to a model server) run any importable callable. Only these classes -- plus any the serving
# process itself adds with register_servable_class() -- are ever imported by LoadedModel.
_SERVABLE = {
    "mifx.models.cnn:FashionCNN",
    "mifx.models.cnn:TpuMnistCNN",
    "mifx.models.cnn:MnistDPCNN",
    "mifx.models.taxi_dnn:TaxiDNN",
    "mifx.models.resnet:ResNetV2",
    "mifx.models.wide_deep:WideDeepModel",
    "torch.nn:Linear",
}


def register_servable_class(class_path: str) -> None:
    """Allow exports naming `module:Class` (an nn.Module subclass) to be loaded by this process."""
    _SERVABLE.add(class_path)


def servable_classes() -> frozenset:
    return frozenset(_SERVABLE)


def _json_plain(v, depth: int = 0) -> bool:
    if depth > 8:
        return False
    if v is None or isinstance(v, (bool, int, float, str)):
        return True
    if isinstance(v, list):
        return all(_json_plain(x, depth + 1) for x in v)
    if isinstance(v, dict):
        return all(isinstance(k, str) and _json_plain(x, depth + 1) for k, x in v.items())
    return False


def _import(path: str):
    if path not in _SERVABLE:
        raise PermissionError(f"model class {path!r} is not servable (allowed: {sorted(_SERVABLE)}; "
                              "register_servable_class() adds one)")
    mod, _, name = path.partition(":")
    cls = getattr(importlib.import_module(mod), name)
    if not (isinstance(cls, type) and issubclass(cls, torch.nn.Module)):
        raise PermissionError(f"model class {path!r} is not a torch.nn.Module")
    return cls


class LoadedModel:
    def __init__(self, path: str, device: str | None = None):
        self.path = path
        with open(os.path.join(path, "saved_model.json")) as f:
            self.meta = json.load(f)
        if self.meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a {FORMAT} export")
        self.device = torch.device(device) if device else (torch.device("cuda") if torch.cuda.is_available()
                                                          else torch.device("cpu"))
        sd = load_file(os.path.join(path, "variables", "variables.safetensors"))
        self.family = self.meta["family"]
        self.transform = None
        if self.family not in ("wide_deep", "module"):
            raise ValueError(f"{path}: unknown model family {self.family!r}")
        if self.family == "wide_deep":
            from ..models import wide_deep as wdm

            mc = self.meta["model_config"]
            cfg = wdm.WideDeepConfig(dense_features=mc["dense_features"], wide=[tuple(x) for x in mc["wide"]],
                                     hidden_units=mc["hidden_units"], label=mc["label"])
            self.model = wdm.WideDeepModel(cfg, seed=None)
            self.model.load_state_dict(sd, strict=False)
            tdir = os.path.join(path, "assets", "transform")
            if self.meta["receiver"].get("has_transform") and os.path.isdir(tdir):
                from ..transform import TransformOutput

                self.transform = TransformOutput(tdir)
            self._fused = None
        else:
            cls = _import(self.meta["model_class"])
            cfg = self.meta.get("model_config", {})
            if not (isinstance(cfg, dict) and _json_plain(cfg)):
                raise ValueError(f"{path}: model_config must be a JSON object of plain values")
            self.model = cls(**cfg)
            self.model.load_state_dict(sd)
            self.model.to(self.device).eval()

    @property
    def signatures(self) -> dict:
        return self.meta["signatures"]

    # ------------------------------------------------------------------ wide & deep
    def _wd_records(self, columns: dict, with_label: bool) -> np.ndarray:
        from ..models import wide_deep as wdm

        cols = self.transform.transform_raw_features(columns) if self.transform else columns
        return wdm.pack_transformed_columns(cols, self.model.cfg, with_label=with_label)

    def wd_logits(self, columns: dict) -> np.ndarray:
        from ..models import wide_deep as wdm

        rec = self._wd_records(columns, with_label=False)
        t = torch.from_numpy(rec.view(np.uint8).reshape(-1, 32).copy())
        if self.device.type == "cuda" and len(rec):
            if self._fused is None:
                from ..trainer.fused_wide_deep import FusedWideDeepTrainer

                self._fused = FusedWideDeepTrainer(self.model, batch=64, device=self.device)
            return self._fused.predict_logits(t).cpu().numpy()
        dense, ids, _ = wdm.records_to_tensors(t)
        with torch.no_grad():
            return self.model(dense, ids).numpy()

    def predict(self, instances) -> dict:
        """instances: list of feature dicts (TF-Serving row format) or dict of columns."""
        if self.family == "wide_deep":
            if isinstance(instances, list):
                keys = sorted({k for r in instances for k in r})
                columns = {k: np.array([r.get(k) for r in instances], dtype=object) for k in keys}
                for k, v in columns.items():
                    if all(isinstance(x, (int, float)) or x is None for x in v):
                        if any(isinstance(x, float) for x in v):
                            columns[k] = np.array([np.nan if x is None else x for x in v], dtype=np.float64)
            else:
                columns = instances
            logits = self.wd_logits(columns)
            p = 1.0 / (1.0 + np.exp(-logits))
            cls = (p > 0.5).astype(np.int64)
            return {"logits": logits[:, None], "logistic": p[:, None], "probabilities": np.stack([1 - p, p], 1),
                    "class_ids": cls[:, None], "classes": cls.astype(str)[:, None]}
        x = torch.as_tensor(np.asarray(instances, dtype=np.float32), device=self.device)
        with torch.no_grad():
            return {"scores": self.model(x).float().cpu().numpy()}


def load(path: str, device: str | None = None) -> LoadedModel:
    return LoadedModel(path, device)


def latest_export(export_dir_base: str) -> str:
    vs = [d for d in os.listdir(export_dir_base) if d.isdigit()]
    if not vs:
        raise FileNotFoundError(f"no versioned exports under {export_dir_base}")
    return os.path.join(export_dir_base, max(vs, key=int))
